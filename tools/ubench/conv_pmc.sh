# PMC passes over the standalone conv kernels (tools/ubench/convbench.py), one counter group per run.
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
run() {
  d=$1; shift
  rm -rf $R/gpurun_out/$d
  timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d $R/gpurun_out/$d -- python3 $R/tools/ubench/convbench.py --iters 3 > $R/gpurun_out/$d.log 2>&1
}
run cpmcA SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE && \
run cpmcB SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM GRBM_GUI_ACTIVE && \
run cpmcC SQ_INSTS_SALU SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM SQ_WAVES SQ_INSTS_SMEM SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE
echo rc=$?
