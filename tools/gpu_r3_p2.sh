# Round 3 step P2: critical path on a high-priority stream (PBX_MAIN_PRIO=1) vs default, same box; host micro-optimisations in
R=$GRAFT_REPO_ROOT
cd $R
T="timeout -k 10"
$T 300 python -u -m pytest tests/test_graph_step.py tests/test_gpu_ddp_streams.py -x -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r3p2_tests.log 2>&1 || { tail -30 gpurun_out/r3p2_tests.log; exit 1; }
tail -1 gpurun_out/r3p2_tests.log
for i in 1 2 3; do
  for v in 1 0; do PBX_MAIN_PRIO=$v $T 300 python -u bench.py > gpurun_out/r3p2_bench_p${v}_$i.json 2> gpurun_out/r3p2_bench_p${v}_$i.err || exit 1; python3 -c "import json;d=json.load(open('gpurun_out/r3p2_bench_p${v}_$i.json'));print('main_prio=$v',d['value'],d['ms_per_step'])"; done
done
$T 300 python -u tools/cpu_overhead.py --steps 30 2>&1 | grep issue
