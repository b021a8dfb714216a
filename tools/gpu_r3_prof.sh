# Final-tree kernel trace of the headline step: per-kernel stats and the two-stream critical path
R=$GRAFT_REPO_ROOT
cd $R
T="timeout -k 10"
O=gpurun_out/r3_prof
mkdir -p $O
$T 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/conc -- python3 $R/bench.py --steps 5 --warmup 3 > $O/conc.log 2>&1 || { tail -20 $O/conc.log; exit 1; }
s=$(find $O/conc -name '*kernel_stats.csv' | head -1); python3 tools/profsum.py $s 8 > $O/kernel_summary.txt
t=$(find $O/conc -name '*kernel_trace.csv' | head -1); python3 tools/critpath.py $t 2 > $O/critpath.txt
head -30 $O/kernel_summary.txt
head -12 $O/critpath.txt
