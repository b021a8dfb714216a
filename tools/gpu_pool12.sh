# pool forward with 32-position items / 3 waves per SIMD (PBX_ATTN_FWD2=12) vs the 64-position form (8)
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_hip_local_track.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/p12_tests.log 2>&1 || { tail -40 gpurun_out/p12_tests.log; exit 1; }
tail -1 gpurun_out/p12_tests.log
for c in 8 12; do
  PBX_ATTN_FWD2=$c timeout -k 10 120 python -u tools/ubench/poolbench.py > gpurun_out/p12_pool_$c.log 2>&1 || { cat gpurun_out/p12_pool_$c.log; exit 1; }
  echo "== cfg $c $(grep ln_attn_fwd2 gpurun_out/p12_pool_$c.log)"
done
bash tools/ab_envs.sh 3 "PBX_ATTN_FWD2=8" "PBX_ATTN_FWD2=12"
