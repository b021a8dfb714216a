# Round 3 step HY: hybrid pool backward (PBX_POOL_RECOMPUTE=2: half the columns stored, half recomputed) - numerics, same-box A/B, trace
R=$GRAFT_REPO_ROOT
cd $R
T="timeout -k 10"
$T 600 python -u -m pytest tests/test_hip_local_track.py -x -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r3hy_tests.log 2>&1 || { grep -E "Error|error|assert|FAIL|failed" gpurun_out/r3hy_tests.log | tail -30; exit 1; }
tail -1 gpurun_out/r3hy_tests.log
for i in 1 2 3; do
  for v in 2 0; do PBX_POOL_RECOMPUTE=$v $T 300 python -u bench.py > gpurun_out/r3hy_bench_m${v}_$i.json 2> gpurun_out/r3hy_bench_m${v}_$i.err || exit 1; python3 -c "import json;d=json.load(open('gpurun_out/r3hy_bench_m${v}_$i.json'));print('pool_mode=$v',d['value'],d['ms_per_step'])"; done
done
cd /tmp && export TMPDIR=/tmp
PBX_POOL_RECOMPUTE=2 $T 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r3hy_conc -- python3 $R/bench.py --steps 5 --warmup 3 > $R/gpurun_out/r3hy_conc.log 2>&1 || exit 1
cd $R
s=$(find gpurun_out/r3hy_conc -name '*kernel_stats.csv' | head -1); python3 tools/profsum.py $s 8 > gpurun_out/r3hy_kernel_summary.txt
head -8 gpurun_out/r3hy_kernel_summary.txt; grep -E "attn|ln_attn" gpurun_out/r3hy_kernel_summary.txt
