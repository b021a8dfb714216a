#!/bin/bash
# GELU-core variants of the recompute pool (csrc/pool.hip) on one box: numerics vs fp32 + timing.
# libs from tools/ubench/build_flags.sh: base, fast1 (2-term logistic fwd), fast2 (3-term logistic fwd +
# tanh-form bwd), nogelu (ablation: no GELU / GELU').
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
for v in base fast1 fast2 nogelu base fast2; do
  PBX_HIP_LIB=tools/ubench/abl/libpbx_$v.so timeout -k 10 200 python -u tools/ubench/poolbench.py > gpurun_out/pb_$v.log 2>&1 \
    || { echo "FAIL $v"; tail gpurun_out/pb_$v.log; exit 1; }
  echo "== $v"; grep -v amdgpu.ids gpurun_out/pb_$v.log
done
