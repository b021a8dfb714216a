cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/ubench/poolbench.py > gpurun_out/poolbench2.log 2>&1 || { echo FAIL; cat gpurun_out/poolbench2.log | tail; exit 1; }
cat gpurun_out/poolbench2.log | grep -v amdgpu.ids
rm -rf gpurun_out/pool_pmc
timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU -d gpurun_out/pool_pmc -o run -- python3 -u tools/ubench/poolbench.py --iters 3 > gpurun_out/pool_pmc.log 2>&1 || { echo PMCFAIL; tail gpurun_out/pool_pmc.log; exit 1; }
python3 tools/pmcsum.py pool_pmc
