# Round 3 step H: column-split global track (PBX_GLOB3), local-head fold, head weight grads on the aux
# stream, new GELU cores: numerics + same-box bench A/B + a concurrent trace
R=$GRAFT_REPO_ROOT
cd $R
T="timeout -k 10"
$T 600 python -u -m pytest tests/test_hip_global_track.py tests/test_hip_heads.py tests/test_hip_local_track.py tests/test_determinism.py tests/test_hip_gemm.py -x -q -s --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r3h_tests.log 2>&1 || { grep -E "max \||rel-l2|Error|assert|FAIL" gpurun_out/r3h_tests.log | tail -30; tail -5 gpurun_out/r3h_tests.log; exit 1; }
tail -1 gpurun_out/r3h_tests.log
for i in 1 2; do
  for v in 1 0; do PBX_GLOB3=$v $T 300 python -u bench.py > gpurun_out/r3h_bench_g${v}_$i.json 2> gpurun_out/r3h_bench_g${v}_$i.err || exit 1; python3 -c "import json;d=json.load(open('gpurun_out/r3h_bench_g${v}_$i.json'));print('glob3=$v',d['value'],d['ms_per_step'])"; done
done
PBX_HIP_LIB=$R/tools/ubench/abl/libpbx_oldgelu.so PBX_GLOB3=0 $T 300 python -u bench.py > gpurun_out/r3h_bench_oldgelu.json 2> gpurun_out/r3h_bench_oldgelu.err && python3 -c "import json;d=json.load(open('gpurun_out/r3h_bench_oldgelu.json'));print('oldgelu lib (glob2)',d['value'],d['ms_per_step'])"
cd /tmp && export TMPDIR=/tmp
$T 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r3h_conc -- python3 $R/bench.py --steps 5 --warmup 3 > $R/gpurun_out/r3h_conc.log 2>&1 || exit 1
cd $R
t=$(find gpurun_out/r3h_conc -name '*kernel_trace.csv' | head -1); python3 tools/stepspan.py $t 4 > gpurun_out/r3h_conc_steps.txt; python3 tools/critpath.py $t 2 > gpurun_out/r3h_critpath.txt
head -12 gpurun_out/r3h_conc_steps.txt; head -20 gpurun_out/r3h_critpath.txt
