timeout -k 10 300 python -u -m pytest tests/test_hip_pool.py tests/test_hip_local_track.py tests/test_hip_numerics_elementwise.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t_ep.log 2>&1; tail -2 gpurun_out/t_ep.log
for v in prev cur prev cur; do
  if [ $v = prev ]; then export PBX_HIP_LIB=tools/ubench/abl/libpbx_prev.so; else unset PBX_HIP_LIB; fi
  timeout -k 10 100 python -u tools/ubench/poolbench.py 2>&1 | grep -E "B=1024|numerics" | sed "s/^/$v /"
done
unset PBX_HIP_LIB
PBX_HIP_LIB=tools/ubench/abl/libpbx_stamps.so timeout -k 10 100 python -u tools/ubench/poolstamps.py 2>&1 | grep -v amdgpu.ids
bash tools/gpu.sh ab ep "PBX_HIP_LIB=tools/ubench/abl/libpbx_prev.so" "PBX_X=0" 3 --steps 30
