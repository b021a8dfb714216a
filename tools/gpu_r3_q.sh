# Round 3 step Q: sparse input layer with its W^T image / CSC on an aux stream; full-chip conv weight gradient for the last block
R=$GRAFT_REPO_ROOT
cd $R
T="timeout -k 10"
$T 600 python -u -m pytest tests/test_hip_input_layer.py tests/test_hip_local_track.py tests/test_determinism.py tests/test_graph_step.py tests/test_gpu_ddp_streams.py -x -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r3q_tests.log 2>&1 || { grep -E "Error|assert|FAIL|failed" gpurun_out/r3q_tests.log | tail -30; exit 1; }
tail -1 gpurun_out/r3q_tests.log
for i in 1 2 3; do
  for v in "1 1" "1 0" "0 0"; do set -- $v; PBX_WGRAD_TAIL_FULL=$1 PBX_ANN_SPARSE=$2 $T 300 python -u bench.py > gpurun_out/r3q_bench_t$1s$2_$i.json 2> gpurun_out/r3q_bench_t$1s$2_$i.err || exit 1; python3 -c "import json;d=json.load(open('gpurun_out/r3q_bench_t$1s$2_$i.json'));print('tail_full=$1 ann_sparse=$2',d['value'],d['ms_per_step'])"; done
done
cd /tmp && export TMPDIR=/tmp
$T 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r3q_conc -- python3 $R/bench.py --steps 5 --warmup 3 > $R/gpurun_out/r3q_conc.log 2>&1 || exit 1
cd $R
t=$(find gpurun_out/r3q_conc -name '*kernel_trace.csv' | head -1); python3 tools/critpath.py $t 2 > gpurun_out/r3q_critpath.txt
head -4 gpurun_out/r3q_critpath.txt; tail -14 gpurun_out/r3q_critpath.txt
