# Round 3: host cost of the aux-stream hand-offs (cached events + set_stream, PBX_STREAM_FAST=1) vs per-call events +
# stream contexts (0): stream / graph / DP tests, host issue time and bench, same box
R=$GRAFT_REPO_ROOT
cd $R
T="timeout -k 10"
$T 600 python -u -m pytest tests/test_graph_step.py tests/test_gpu_ddp_streams.py tests/test_gpu_dp_multirank.py tests/test_hip_local_track.py tests/test_hip_input_layer.py tests/test_determinism.py -x -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r3sf_tests.log 2>&1 || { grep -E "Error|error|assert|FAIL|failed" gpurun_out/r3sf_tests.log | tail -30; exit 1; }
tail -1 gpurun_out/r3sf_tests.log
for i in 1 2 3; do
  for v in 1 0; do
    PBX_STREAM_FAST=$v $T 300 python -u tools/host_breakdown.py --steps 30 2>&1 | grep issue | sed "s/^/fast=$v /"
    PBX_STREAM_FAST=$v $T 300 python -u bench.py > gpurun_out/r3sf_bench_f${v}_$i.json 2> gpurun_out/r3sf_bench_f${v}_$i.err || exit 1
    python3 -c "import json;d=json.load(open('gpurun_out/r3sf_bench_f${v}_$i.json'));print('fast=$v bench',d['value'],d['ms_per_step'])"
  done
done
