# Round 3 step V: local-MLP weight-gradient folds on the aux stream - tests, same-box A/B, trace
R=$GRAFT_REPO_ROOT
cd $R
T="timeout -k 10"
$T 600 python -u -m pytest tests/test_hip_local_track.py tests/test_determinism.py tests/test_graph_step.py tests/test_gpu_ddp_streams.py tests/test_gpu_dp_multirank.py -x -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r3v_tests.log 2>&1 || { grep -E "Error|assert|FAIL|failed" gpurun_out/r3v_tests.log | tail -30; exit 1; }
tail -1 gpurun_out/r3v_tests.log
for i in 1 2 3; do
  for v in 1 0; do PBX_LN2_LATE_FOLD=$v $T 300 python -u bench.py > gpurun_out/r3v_bench_f${v}_$i.json 2> gpurun_out/r3v_bench_f${v}_$i.err || exit 1; python3 -c "import json;d=json.load(open('gpurun_out/r3v_bench_f${v}_$i.json'));print('ln2_late_fold=$v',d['value'],d['ms_per_step'])"; done
done
cd /tmp && export TMPDIR=/tmp
$T 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r3v_conc -- python3 $R/bench.py --steps 5 --warmup 3 > $R/gpurun_out/r3v_conc.log 2>&1 || exit 1
cd $R
t=$(find gpurun_out/r3v_conc -name '*kernel_trace.csv' | head -1); python3 tools/critpath.py $t 2 > gpurun_out/r3v_critpath.txt
s=$(find gpurun_out/r3v_conc -name '*kernel_stats.csv' | head -1); python3 tools/profsum.py $s 8 > gpurun_out/r3v_kernel_summary.txt
head -4 gpurun_out/r3v_critpath.txt
