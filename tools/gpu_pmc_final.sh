# Round-1 final: ZeRO GPU test, then PMC passes over the L=512 B=512 bench (eager launches, 2 steps),
# one counter group per rocprofv3 run (SQ <= 8, TCC <= 4 per pass).
R=$GRAFT_REPO_ROOT
cd $R && timeout -k 10 200 python -u -m pytest tests/test_zero.py -m gpu -x -v --timeout 120 --timeout-method thread > $R/gpurun_out/r1_v16_zero_gpu.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
run() {  # $1 = out dir name, rest = counters
  d=$1; shift
  rm -rf $R/gpurun_out/$d
  timeout -s KILL 150 rocprofv3 --pmc "$@" --output-format csv -d $R/gpurun_out/$d -- python3 $R/bench.py --steps 2 --warmup 1 > $R/gpurun_out/$d.log 2>&1
}
run pmcA SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE && \
run pmcB SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM GRBM_GUI_ACTIVE && \
run pmcC TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE
echo rc=$?
