# Round 3 step LF:  LN1/MLP forward with two samples of s1 in flight vs one
# (HEAD library as PBX_HIP_LIB=tools/ubench/abl/libpbx_base.so) - numerics, same-box A/B, serial kernel time
R=$GRAFT_REPO_ROOT
cd $R
T="timeout -k 10"
$T 600 python -u -m pytest tests/test_hip_local_track.py tests/test_determinism.py -x -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r3lf_tests.log 2>&1 || { grep -E "Error|error|assert|FAIL|failed" gpurun_out/r3lf_tests.log | tail -30; exit 1; }
tail -1 gpurun_out/r3lf_tests.log
for i in 1 2 3; do
  $T 300 python -u bench.py > gpurun_out/r3lf_bench_new_$i.json 2> gpurun_out/r3lf_bench_new_$i.err || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/r3lf_bench_new_$i.json'));print('ln_linear_fwd prefetch2',d['value'],d['ms_per_step'])"
  PBX_HIP_LIB=tools/ubench/abl/libpbx_base.so $T 300 python -u bench.py > gpurun_out/r3lf_bench_base_$i.json 2> gpurun_out/r3lf_bench_base_$i.err || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/r3lf_bench_base_$i.json'));print('ln_linear_fwd base     ',d['value'],d['ms_per_step'])"
done
cd /tmp && export TMPDIR=/tmp
PBX_AUX_STREAM=0 $T 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r3lf_serial -- python3 $R/bench.py --steps 5 --warmup 3 > $R/gpurun_out/r3lf_serial.log 2>&1 || exit 1
cd $R
s=$(find gpurun_out/r3lf_serial -name '*kernel_stats.csv' | head -1); python3 tools/profsum.py $s 8 40 > gpurun_out/r3lf_serial_kernel_summary.txt
grep -E "ln_linear_fwd" gpurun_out/r3lf_serial_kernel_summary.txt
