# Round 3 step L (new session): full GPU suite, smoke, headline bench, host issue cost, concurrent trace
R=$GRAFT_REPO_ROOT
cd $R
T="timeout -k 10"
$T 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r3l_gpu_tests.log 2>&1 || { tail -40 gpurun_out/r3l_gpu_tests.log; exit 1; }
tail -2 gpurun_out/r3l_gpu_tests.log
$T 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3l_smoke.log 2>&1 || { tail -20 gpurun_out/r3l_smoke.log; exit 1; }
tail -1 gpurun_out/r3l_smoke.log
$T 300 python -u bench.py > gpurun_out/r3l_bench_l512.json 2> gpurun_out/r3l_bench_l512.err || exit 1
cat gpurun_out/r3l_bench_l512.json
$T 300 python -u tools/cpu_overhead.py --steps 30 > gpurun_out/r3l_cpu_overhead.txt 2>&1 || exit 1
cat gpurun_out/r3l_cpu_overhead.txt
PBX_CPROFILE=1 $T 300 python -u tools/cpu_overhead.py --steps 10 > gpurun_out/r3l_cpu_cprofile.txt 2>&1 || exit 1
