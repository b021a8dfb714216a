# packed vs scalar f32 GELU cores beside MFMAs: pool / LN / conv kernels standalone, then the step
cd $GRAFT_REPO_ROOT
for v in cur scal noslp; do
  if [ $v = cur ]; then lib=""; else lib=tools/ubench/abl/libpbx_$v.so; fi
  PBX_HIP_LIB=$lib timeout -k 10 120 python -u tools/ubench/poolbench.py > gpurun_out/sab_pool_$v.log 2>&1 || { cat gpurun_out/sab_pool_$v.log; exit 1; }
  PBX_HIP_LIB=$lib timeout -k 10 120 python -u tools/ubench/convbench.py > gpurun_out/sab_conv_$v.log 2>&1 || { cat gpurun_out/sab_conv_$v.log; exit 1; }
  echo "== $v"; cat gpurun_out/sab_pool_$v.log gpurun_out/sab_conv_$v.log | grep -v Warn
done
for r in 1 2; do for v in cur scal noslp; do
  if [ $v = cur ]; then lib=""; else lib=tools/ubench/abl/libpbx_$v.so; fi
  PBX_HIP_LIB=$lib timeout -k 10 200 python -u bench.py --steps 30 > gpurun_out/sab_bench_${v}_$r.json 2>/dev/null || exit 1
  echo "bench $v run $r: $(python3 -c "import json;d=json.load(open('gpurun_out/sab_bench_${v}_$r.json'));print(d['value'], d['ms_per_step'])")"
done; done
