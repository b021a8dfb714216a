# PMC passes over the paper-semantics bench step (one counter group per rocprofv3 run)
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
run() {  # $1 = out dir name, rest = counters
  d=$1; shift
  rm -rf $R/gpurun_out/$d
  timeout -s KILL 150 rocprofv3 --pmc "$@" --output-format csv -d $R/gpurun_out/$d -- python3 $R/bench.py --semantics paper --steps 2 --warmup 1 > $R/gpurun_out/$d.log 2>&1
}
run ppA SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE && \
run ppB SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM GRBM_GUI_ACTIVE
echo rc=$?
