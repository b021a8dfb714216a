# Round 3 step I: global-track backward one-launch vs column-split (forward split in both), same box
R=$GRAFT_REPO_ROOT
cd $R
T="timeout -k 10"
$T 600 python -u -m pytest tests/test_hip_global_track.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r3i_tests.log 2>&1 || { tail -30 gpurun_out/r3i_tests.log; exit 1; }
tail -1 gpurun_out/r3i_tests.log
for i in 1 2 3; do
  for v in 0 1; do PBX_GLOB3_BWD=$v $T 300 python -u bench.py > gpurun_out/r3i_bench_b${v}_$i.json 2> gpurun_out/r3i_bench_b${v}_$i.err || exit 1; python3 -c "import json;d=json.load(open('gpurun_out/r3i_bench_b${v}_$i.json'));print('glob3_bwd=$v',d['value'],d['ms_per_step'])"; done
done
