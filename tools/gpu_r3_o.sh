# Round 3 step O: global-track backward on a high-priority aux stream (beside the conv data gradient), same-box A/B
R=$GRAFT_REPO_ROOT
cd $R
T="timeout -k 10"
$T 300 python -u -m pytest tests/test_gpu_ddp_streams.py tests/test_hip_global_track.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r3o_tests_default.log 2>&1 || { tail -30 gpurun_out/r3o_tests_default.log; exit 1; }
PBX_GLOBAL_STREAM=1 PBX_GLOBAL_PRIO=1 $T 300 python -u -m pytest tests/test_gpu_ddp_streams.py tests/test_hip_local_track.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r3o_tests_gprio.log 2>&1 || { tail -30 gpurun_out/r3o_tests_gprio.log; exit 1; }
tail -1 gpurun_out/r3o_tests_gprio.log
for i in 1 2 3; do
  for v in "0 0" "1 1" "1 0"; do set -- $v; PBX_GLOBAL_STREAM=$1 PBX_GLOBAL_PRIO=$2 $T 300 python -u bench.py > gpurun_out/r3o_bench_g$1p$2_$i.json 2> gpurun_out/r3o_bench_g$1p$2_$i.err || exit 1; python3 -c "import json;d=json.load(open('gpurun_out/r3o_bench_g$1p$2_$i.json'));print('global_stream=$1 prio=$2',d['value'],d['ms_per_step'])"; done
done
cd /tmp && export TMPDIR=/tmp
PBX_GLOBAL_STREAM=1 PBX_GLOBAL_PRIO=1 $T 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r3o_conc -- python3 $R/bench.py --steps 5 --warmup 3 > $R/gpurun_out/r3o_conc.log 2>&1 || exit 1
cd $R
t=$(find gpurun_out/r3o_conc -name '*kernel_trace.csv' | head -1); python3 tools/critpath.py $t 2 > gpurun_out/r3o_critpath.txt
head -12 gpurun_out/r3o_critpath.txt
