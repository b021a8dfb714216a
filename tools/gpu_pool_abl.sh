# attention-pool forward ablations: GELU chains off, GELU' fragment stores off, both
cd $GRAFT_REPO_ROOT
for v in cur nogelu nogstore noboth; do
  if [ $v = cur ]; then lib=""; else lib=tools/ubench/abl/libpbx_$v.so; fi
  PBX_HIP_LIB=$lib timeout -k 10 120 python -u tools/ubench/poolbench.py > gpurun_out/poolabl_$v.log 2>&1 || { cat gpurun_out/poolabl_$v.log; exit 1; }
  echo "== $v"; grep -E "attn" gpurun_out/poolabl_$v.log
done
