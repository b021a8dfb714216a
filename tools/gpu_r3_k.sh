# Round 3 step K: one-launch local head (PBX_LHEAD_FUSED) - numerics, same-box bench A/B, trace
R=$GRAFT_REPO_ROOT
cd $R
T="timeout -k 10"
$T 600 python -u -m pytest tests/test_hip_heads.py tests/test_hip_local_track.py -x -q -s --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r3k_tests.log 2>&1 || { grep -E "err|Error|assert" gpurun_out/r3k_tests.log | tail -30; exit 1; }
tail -1 gpurun_out/r3k_tests.log
for i in 1 2 3; do
  for v in 1 0; do PBX_LHEAD_FUSED=$v PBX_ATTN_FIXTW=$v $T 300 python -u bench.py > gpurun_out/r3k_bench_f${v}_$i.json 2> gpurun_out/r3k_bench_f${v}_$i.err || exit 1; python3 -c "import json;d=json.load(open('gpurun_out/r3k_bench_f${v}_$i.json'));print('lhead_fused+attn_fixtw=$v',d['value'],d['ms_per_step'])"; done
done
cd /tmp && export TMPDIR=/tmp
$T 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r3k_conc -- python3 $R/bench.py --steps 5 --warmup 3 > $R/gpurun_out/r3k_conc.log 2>&1 || exit 1
cd $R
t=$(find gpurun_out/r3k_conc -name '*kernel_trace.csv' | head -1); python3 tools/critpath.py $t 2 > gpurun_out/r3k_critpath.txt
grep -E "lhead|span|queue" gpurun_out/r3k_critpath.txt | head -12
