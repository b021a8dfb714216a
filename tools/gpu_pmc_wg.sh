# PMC passes over the weight-gradient kernel alone (tools/wgbench.py)
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
run() {  # $1 = out dir name, rest = counters
  d=$1; shift
  rm -rf $R/gpurun_out/$d
  timeout -s KILL 90 rocprofv3 --pmc "$@" --output-format csv -d $R/gpurun_out/$d -- python3 $R/tools/wgbench.py > $R/gpurun_out/$d.log 2>&1
}
run wgA SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE && \
run wgB SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE && \
timeout -s KILL 90 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/wgT -- python3 $R/tools/wgbench.py > $R/gpurun_out/wgT.log 2>&1
echo rc=$?
