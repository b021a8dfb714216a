# conv forward / data gradient: XCD-aware tile remap (abl build "xcd") vs the tree build
cd $GRAFT_REPO_ROOT
PBX_HIP_LIB=tools/ubench/abl/libpbx_xcd.so timeout -k 10 400 python -u -m pytest tests/test_hip_local_track.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/xcd_tests.log 2>&1 || { tail -40 gpurun_out/xcd_tests.log; exit 1; }
tail -1 gpurun_out/xcd_tests.log
for v in cur; do
  if [ $v = cur ]; then lib=""; else lib=tools/ubench/abl/libpbx_$v.so; fi
  PBX_HIP_LIB=$lib timeout -k 10 120 python -u tools/ubench/convbench.py > gpurun_out/xcd_conv_$v.log 2>&1 || { cat gpurun_out/xcd_conv_$v.log; exit 1; }
  echo "== $v"; grep conv_ gpurun_out/xcd_conv_$v.log
done
for r in 1 2 3; do for v in cur; do
  if [ $v = cur ]; then lib=""; else lib=tools/ubench/abl/libpbx_$v.so; fi
  PBX_HIP_LIB=$lib timeout -k 10 200 python -u bench.py --steps 30 > gpurun_out/xcd_bench_${v}_$r.json 2>/dev/null || exit 1
  echo "bench $v run $r: $(python3 -c "import json;d=json.load(open('gpurun_out/xcd_bench_${v}_$r.json'));print(d['value'], d['ms_per_step'])")"
done; done
