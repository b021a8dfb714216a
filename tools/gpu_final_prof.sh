# End-of-round evidence: serial kernel stats (every kernel on the main stream) and one PMC pass over
# the headline bench.
R=$GRAFT_REPO_ROOT
bash $R/tools/gpu_prof_serial.sh r2_final_serial || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU GRBM_GUI_ACTIVE --output-format csv -d $R/gpurun_out/r2_final_pmcA -- python3 $R/bench.py --steps 2 --warmup 1 > $R/gpurun_out/r2_final_pmcA.log 2>&1
echo rc=$?
