# Phase ablation of the conv kernels: each variant is a separate build (tools/ubench/build_flags.sh).
R=$GRAFT_REPO_ROOT
cd $R
for v in "$@"; do
  PBX_HIP_LIB=tools/ubench/abl/libpbx_$v.so timeout -k 10 120 python -u tools/ubench/convbench.py --tag $v >> gpurun_out/convab.log 2>&1 || exit 1
done
