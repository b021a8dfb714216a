cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 60 ./tools/ubench/valu_rate > gpurun_out/valu_rate.log 2>&1 || { echo VALUFAIL; cat gpurun_out/valu_rate.log; exit 1; }
cat gpurun_out/valu_rate.log
timeout -k 10 200 python -u tools/ubench/poolbench.py > gpurun_out/pb_base.log 2>&1 || { echo FAIL; tail gpurun_out/pb_base.log; exit 1; }
grep -v amdgpu.ids gpurun_out/pb_base.log
PBX_HIP_LIB=tools/ubench/abl/libpbx_tanh.so timeout -k 10 200 python -u tools/ubench/poolbench.py > gpurun_out/pb_tanh.log 2>&1 || { echo FAIL; tail gpurun_out/pb_tanh.log; exit 1; }
grep -v amdgpu.ids gpurun_out/pb_tanh.log
