# Round 3 step D: GEMM / heads numerics after the split-K + GO-epilogue rework, serial and concurrent
# kernel traces, headline bench.
R=$GRAFT_REPO_ROOT
cd $R
T="timeout -k 10"
$T 400 python -u -m pytest tests/test_hip_gemm.py tests/test_hip_heads.py tests/test_determinism.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r3d_tests.log 2>&1 || { tail -40 gpurun_out/r3d_tests.log; exit 1; }
tail -2 gpurun_out/r3d_tests.log
$T 200 python -u tools/gemm_ubench_cold.py > gpurun_out/r3d_gemm_cold.txt 2>&1 || exit 1
cat gpurun_out/r3d_gemm_cold.txt
$T 300 python -u bench.py > gpurun_out/r3d_bench.json 2> gpurun_out/r3d_bench.err || exit 1
cat gpurun_out/r3d_bench.json
bash $R/tools/gpu_prof_serial.sh r3d_serial || exit 1
f=$(find gpurun_out/r3d_serial -name '*kernel_stats.csv' | head -1); python3 tools/profsum.py $f 8 40 > gpurun_out/r3d_serial_summary.txt
head -25 gpurun_out/r3d_serial_summary.txt
cd /tmp && export TMPDIR=/tmp
$T 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r3d_conc -- python3 $R/bench.py --steps 5 --warmup 3 > $R/gpurun_out/r3d_conc.log 2>&1 || exit 1
cd $R
t=$(find gpurun_out/r3d_conc -name '*kernel_trace.csv' | head -1); python3 tools/stepspan.py $t 4 > gpurun_out/r3d_conc_steps.txt
head -24 gpurun_out/r3d_conc_steps.txt
