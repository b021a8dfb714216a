# standalone pool / LN kernel timings: current build vs the no-GELU ablation build
cd $GRAFT_REPO_ROOT
timeout -k 10 120 python -u tools/ubench/poolbench.py > gpurun_out/poolb_cur.log 2>&1 || { cat gpurun_out/poolb_cur.log; exit 1; }
PBX_HIP_LIB=tools/ubench/abl/libpbx_nogelu.so timeout -k 10 120 python -u tools/ubench/poolbench.py > gpurun_out/poolb_nogelu.log 2>&1 || { cat gpurun_out/poolb_nogelu.log; exit 1; }
echo "== current"; cat gpurun_out/poolb_cur.log; echo "== no GELU"; cat gpurun_out/poolb_nogelu.log
