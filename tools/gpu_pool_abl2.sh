# attention-pool forward: time vs batch (start-up / tail share) for the current and no-GELU/no-store builds
cd $GRAFT_REPO_ROOT
for v in cur noboth; do
  if [ $v = cur ]; then lib=""; else lib=tools/ubench/abl/libpbx_$v.so; fi
  for B in 128 256 512 1024; do
    PBX_HIP_LIB=$lib timeout -k 10 120 python -u tools/ubench/poolbench.py --B $B > gpurun_out/poolabl2_${v}_$B.log 2>&1 || { cat gpurun_out/poolabl2_${v}_$B.log; exit 1; }
    echo "== $v B=$B $(grep -E 'ln_attn_fwd2' gpurun_out/poolabl2_${v}_$B.log)"
  done
done
