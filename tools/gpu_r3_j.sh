# Round 3 step J: deferred conv weight gradient (PBX_WGRAD_DEFER) - DP/stream tests + same-box A/B
R=$GRAFT_REPO_ROOT
cd $R
T="timeout -k 10"
$T 600 python -u -m pytest tests/test_gpu_ddp_streams.py tests/test_hip_local_track.py tests/test_gpu_dp_multirank.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r3j_tests.log 2>&1 || { tail -30 gpurun_out/r3j_tests.log; exit 1; }
tail -1 gpurun_out/r3j_tests.log
for i in 1 2 3; do
  for v in 1 0; do PBX_WGRAD_DEFER=$v $T 300 python -u bench.py > gpurun_out/r3j_bench_d${v}_$i.json 2> gpurun_out/r3j_bench_d${v}_$i.err || exit 1; python3 -c "import json;d=json.load(open('gpurun_out/r3j_bench_d${v}_$i.json'));print('defer=$v',d['value'],d['ms_per_step'])"; done
done
cd /tmp && export TMPDIR=/tmp
$T 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r3j_conc -- python3 $R/bench.py --steps 5 --warmup 3 > $R/gpurun_out/r3j_conc.log 2>&1 || exit 1
cd $R
t=$(find gpurun_out/r3j_conc -name '*kernel_trace.csv' | head -1); python3 tools/critpath.py $t 2 > gpurun_out/r3j_critpath.txt
head -8 gpurun_out/r3j_critpath.txt
