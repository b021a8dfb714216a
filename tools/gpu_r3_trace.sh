# Round 3 final tree: concurrent and serial (PBX_AUX_STREAM=0) kernel traces of the headline step
R=$GRAFT_REPO_ROOT
T="timeout -k 10"
cd /tmp && export TMPDIR=/tmp
$T 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r3f_conc -- python3 $R/bench.py --steps 5 --warmup 3 > $R/gpurun_out/r3f_conc.log 2>&1 || exit 1
PBX_AUX_STREAM=0 $T 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r3f_serial -- python3 $R/bench.py --steps 5 --warmup 3 > $R/gpurun_out/r3f_serial.log 2>&1 || exit 1
cd $R
t=$(find gpurun_out/r3f_conc -name '*kernel_trace.csv' | head -1); python3 tools/critpath.py $t 2 > gpurun_out/r3f_critpath.txt
s=$(find gpurun_out/r3f_conc -name '*kernel_stats.csv' | head -1); python3 tools/profsum.py $s 8 40 > gpurun_out/r3f_concurrent_kernel_summary.txt
s=$(find gpurun_out/r3f_serial -name '*kernel_stats.csv' | head -1); python3 tools/profsum.py $s 8 40 > gpurun_out/r3f_serial_kernel_summary.txt
head -20 gpurun_out/r3f_serial_kernel_summary.txt
