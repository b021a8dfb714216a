# Round 3 step DG: conv data gradient with a single-pass prologue (each dS1 row loaded once) vs the per-conv passes
# (HEAD library as PBX_HIP_LIB=tools/ubench/abl/libpbx_base.so) - numerics, same-box A/B, serial kernel time
R=$GRAFT_REPO_ROOT
cd $R
T="timeout -k 10"
$T 600 python -u -m pytest tests/test_hip_local_track.py tests/test_determinism.py -x -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r3dg_tests.log 2>&1 || { grep -E "Error|error|assert|FAIL|failed" gpurun_out/r3dg_tests.log | tail -30; exit 1; }
tail -1 gpurun_out/r3dg_tests.log
for i in 1 2 3; do
  $T 300 python -u bench.py > gpurun_out/r3dg_bench_new_$i.json 2> gpurun_out/r3dg_bench_new_$i.err || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/r3dg_bench_new_$i.json'));print('dgrad one-pass',d['value'],d['ms_per_step'])"
  PBX_HIP_LIB=tools/ubench/abl/libpbx_base.so $T 300 python -u bench.py > gpurun_out/r3dg_bench_base_$i.json 2> gpurun_out/r3dg_bench_base_$i.err || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/r3dg_bench_base_$i.json'));print('dgrad base   ',d['value'],d['ms_per_step'])"
done
cd /tmp && export TMPDIR=/tmp
PBX_AUX_STREAM=0 $T 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r3dg_serial -- python3 $R/bench.py --steps 5 --warmup 3 > $R/gpurun_out/r3dg_serial.log 2>&1 || exit 1
cd $R
s=$(find gpurun_out/r3dg_serial -name '*kernel_stats.csv' | head -1); python3 tools/profsum.py $s 8 40 > gpurun_out/r3dg_serial_kernel_summary.txt
grep -E "dgrad" gpurun_out/r3dg_serial_kernel_summary.txt
