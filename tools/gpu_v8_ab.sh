# round-2 v8 A/B: new default build (-fno-slp-vectorize + scalar conv-forward GELU) vs the no-SLP-only
# build vs the pool static-priority build; conv/local-track GPU tests on the new build first
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_hip_local_track.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/v8_tests.log 2>&1 || { tail -30 gpurun_out/v8_tests.log; exit 1; }
tail -1 gpurun_out/v8_tests.log
for v in new noslp prio; do
  if [ $v = new ]; then lib=""; else lib=tools/ubench/abl/libpbx_$v.so; fi
  PBX_HIP_LIB=$lib timeout -k 10 120 python -u tools/ubench/convbench.py > gpurun_out/v8_conv_$v.log 2>&1 || { cat gpurun_out/v8_conv_$v.log; exit 1; }
  PBX_HIP_LIB=$lib timeout -k 10 120 python -u tools/ubench/poolbench.py > gpurun_out/v8_pool_$v.log 2>&1 || { cat gpurun_out/v8_pool_$v.log; exit 1; }
  echo "== $v $(grep conv_fwd3 gpurun_out/v8_conv_$v.log) | $(grep ln_attn_fwd2 gpurun_out/v8_pool_$v.log)"
done
for r in 1 2 3; do for v in new noslp prio; do
  if [ $v = new ]; then lib=""; else lib=tools/ubench/abl/libpbx_$v.so; fi
  PBX_HIP_LIB=$lib timeout -k 10 200 python -u bench.py --steps 30 > gpurun_out/v8_bench_${v}_$r.json 2>/dev/null || exit 1
  echo "bench $v run $r: $(python3 -c "import json;d=json.load(open('gpurun_out/v8_bench_${v}_$r.json'));print(d['value'], d['ms_per_step'])")"
done; done
