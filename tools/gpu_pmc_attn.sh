cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
rm -rf $R/gpurun_out/pmcA1 $R/gpurun_out/pmcA2 $R/gpurun_out/pmcA3
run() {  # $1 = out dir name, rest = counters
  d=$1; shift
  PBX_ATTN_DBG=$DBG timeout -k 10 200 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d $R/gpurun_out/$d -- python3 $R/tools/kbench_attn.py --iters 3 > $R/gpurun_out/$d.log 2>&1
}
export DBG=23
run pmcA1 SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_WR && \
run pmcA2 SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE && \
run pmcA3 SQ_WAIT_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_ANY SQ_INSTS_BRANCH SQ_BUSY_CYCLES
echo rc=$?
