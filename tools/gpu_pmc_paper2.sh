# One PMC pass over the paper-semantics bench (per-kernel MFMA busy / VALU mix / waits).
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
rm -rf $R/gpurun_out/ppmcA $R/gpurun_out/ppmcB
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU GRBM_GUI_ACTIVE --output-format csv -d $R/gpurun_out/ppmcA -- python3 $R/bench.py --steps 2 --warmup 1 --semantics paper > $R/gpurun_out/ppmcA.log 2>&1 && \
timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE --output-format csv -d $R/gpurun_out/ppmcB -- python3 $R/bench.py --steps 2 --warmup 1 --semantics paper > $R/gpurun_out/ppmcB.log 2>&1
echo rc=$?
