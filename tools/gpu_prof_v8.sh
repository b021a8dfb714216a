# round-2 v8 evidence: serial kernel stats (aux stream off) and a concurrent (default streams) kernel trace
R=$GRAFT_REPO_ROOT
bash $R/tools/gpu_prof_serial.sh r2_v8_serial || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r2_v8_conc -- python3 $R/bench.py --steps 5 --warmup 3 > $R/gpurun_out/r2_v8_conc.log 2>&1 || exit 1
cd $R
f=$(find gpurun_out/r2_v8_serial -name '*kernel_stats.csv' | head -1); python3 tools/profsum.py $f 8 32 > gpurun_out/r2_v8_serial_summary.txt
t=$(find gpurun_out/r2_v8_conc -name '*kernel_trace.csv' | head -1); python3 tools/stepspan.py $t 4 > gpurun_out/r2_v8_conc_steps.txt
head -12 gpurun_out/r2_v8_serial_summary.txt; head -8 gpurun_out/r2_v8_conc_steps.txt
