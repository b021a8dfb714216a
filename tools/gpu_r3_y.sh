# Round 3 step Y: recomputing pool backward at two waves per SIMD (attn_bwd3 NW=8) - numerics, same-box A/B vs stored fragments, trace
R=$GRAFT_REPO_ROOT
cd $R
T="timeout -k 10"
$T 600 python -u -m pytest tests/test_hip_local_track.py -x -q -m gpu -k "backward" --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r3y_tests.log 2>&1 || { grep -E "Error|error|assert|FAIL|failed" gpurun_out/r3y_tests.log | tail -30; exit 1; }
tail -1 gpurun_out/r3y_tests.log
for i in 1 2 3; do
  for v in "1 1" "0 1" "1 0"; do set -- $v; PBX_POOL_RECOMPUTE=$1 PBX_POOL_BWD3_WIDE=$2 $T 300 python -u bench.py > gpurun_out/r3y_bench_r$1w$2_$i.json 2> gpurun_out/r3y_bench_r$1w$2_$i.err || exit 1; python3 -c "import json;d=json.load(open('gpurun_out/r3y_bench_r$1w$2_$i.json'));print('pool_recompute=$1 wide=$2',d['value'],d['ms_per_step'])"; done
done
cd /tmp && export TMPDIR=/tmp
PBX_POOL_RECOMPUTE=1 $T 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r3y_conc -- python3 $R/bench.py --steps 5 --warmup 3 > $R/gpurun_out/r3y_conc.log 2>&1 || exit 1
cd $R
s=$(find gpurun_out/r3y_conc -name '*kernel_stats.csv' | head -1); python3 tools/profsum.py $s 8 > gpurun_out/r3y_kernel_summary.txt
head -8 gpurun_out/r3y_kernel_summary.txt
