# Round 3 step W: input-layer backward beside the first block's conv data gradient ("ann" stream) - tests, same-box A/B, DP timeline
R=$GRAFT_REPO_ROOT
cd $R
T="timeout -k 10"
$T 600 python -u -m pytest tests/test_hip_local_track.py tests/test_hip_input_layer.py tests/test_determinism.py tests/test_graph_step.py tests/test_gpu_ddp_streams.py tests/test_gpu_dp_multirank.py -x -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r3w_tests.log 2>&1 || { grep -E "Error|assert|FAIL|failed" gpurun_out/r3w_tests.log | tail -30; exit 1; }
tail -1 gpurun_out/r3w_tests.log
for i in 1 2 3; do
  for v in 1 0; do PBX_INPUT_BWD_EARLY=$v $T 300 python -u bench.py > gpurun_out/r3w_bench_e${v}_$i.json 2> gpurun_out/r3w_bench_e${v}_$i.err || exit 1; python3 -c "import json;d=json.load(open('gpurun_out/r3w_bench_e${v}_$i.json'));print('input_bwd_early=$v',d['value'],d['ms_per_step'])"; done
done
$T 300 python3 tools/dp_timeline.py --steps 6 > gpurun_out/r3w_dp_timeline.txt 2>&1 || { tail -20 gpurun_out/r3w_dp_timeline.txt; exit 1; }
grep -E "bucket|backward|step" gpurun_out/r3w_dp_timeline.txt
