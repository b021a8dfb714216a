# Round 3 step T: PMC passes over the L=512 B=512 headline step (2 steps), one counter group per run (as tools/gpu_pmc_v8.sh)
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
run() {  # $1 = out dir name, rest = counters
  d=$1; shift
  rm -rf $R/gpurun_out/$d
  timeout -s KILL 150 rocprofv3 --pmc "$@" --output-format csv -d $R/gpurun_out/$d -- python3 $R/bench.py --steps 2 --warmup 1 > $R/gpurun_out/$d.log 2>&1
}
run r3pmcA SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE && \
run r3pmcB SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INSTS_SALU GRBM_GUI_ACTIVE && \
run r3bytesF FETCH_SIZE GRBM_GUI_ACTIVE && run r3bytesW WRITE_SIZE GRBM_GUI_ACTIVE
rc=$?
echo rc=$rc
cd $R && python3 tools/pmcsum.py r3pmcA r3pmcB r3bytesF r3bytesW > gpurun_out/r3t_pmc_summary.txt 2>&1; grep -E "attn|conv|wgrad2_kernel|ln_linear|ln2_linear|glob" gpurun_out/r3t_pmc_summary.txt | head -20
exit $rc
