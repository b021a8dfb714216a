# Round 3 step X: recomputing pool backward (attn_bwd3, PBX_POOL_RECOMPUTE) + early input-layer backward (PBX_INPUT_BWD_EARLY):
# numerics vs fp32 torch in both pool modes, same-box A/B, trace, DP timeline
R=$GRAFT_REPO_ROOT
cd $R
T="timeout -k 10"
$T 600 python -u -m pytest tests/test_hip_local_track.py tests/test_graph_step.py -x -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r3x_tests_recompute.log 2>&1 || { grep -E "Error|error|assert|FAIL|failed" gpurun_out/r3x_tests_recompute.log | tail -30; exit 1; }
tail -1 gpurun_out/r3x_tests_recompute.log
PBX_POOL_RECOMPUTE=0 $T 600 python -u -m pytest tests/test_hip_local_track.py -x -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r3x_tests_stored.log 2>&1 || { grep -E "Error|error|assert|FAIL|failed" gpurun_out/r3x_tests_stored.log | tail -30; exit 1; }
tail -1 gpurun_out/r3x_tests_stored.log
$T 600 python -u -m pytest tests/test_hip_input_layer.py tests/test_determinism.py tests/test_graph_step.py tests/test_gpu_ddp_streams.py tests/test_gpu_dp_multirank.py -x -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r3x_tests.log 2>&1 || { grep -E "Error|error|assert|FAIL|failed" gpurun_out/r3x_tests.log | tail -30; exit 1; }
tail -1 gpurun_out/r3x_tests.log
for i in 1 2 3; do
  for v in "1 1" "0 1" "1 0"; do set -- $v; PBX_POOL_RECOMPUTE=$1 PBX_INPUT_BWD_EARLY=$2 $T 300 python -u bench.py > gpurun_out/r3x_bench_r$1e$2_$i.json 2> gpurun_out/r3x_bench_r$1e$2_$i.err || exit 1; python3 -c "import json;d=json.load(open('gpurun_out/r3x_bench_r$1e$2_$i.json'));print('pool_recompute=$1 input_bwd_early=$2',d['value'],d['ms_per_step'])"; done
done
cd /tmp && export TMPDIR=/tmp
$T 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r3x_conc -- python3 $R/bench.py --steps 5 --warmup 3 > $R/gpurun_out/r3x_conc.log 2>&1 || exit 1
cd $R
t=$(find gpurun_out/r3x_conc -name '*kernel_trace.csv' | head -1); python3 tools/critpath.py $t 2 > gpurun_out/r3x_critpath.txt
s=$(find gpurun_out/r3x_conc -name '*kernel_stats.csv' | head -1); python3 tools/profsum.py $s 8 > gpurun_out/r3x_kernel_summary.txt
head -12 gpurun_out/r3x_kernel_summary.txt
$T 300 python3 tools/dp_timeline.py --steps 6 > gpurun_out/r3x_dp_timeline.txt 2>&1 || { tail -20 gpurun_out/r3x_dp_timeline.txt; exit 1; }
grep -E "bucket|backward|step" gpurun_out/r3x_dp_timeline.txt
