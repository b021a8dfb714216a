# Round 3 step S: data-parallel overlap timeline on one GPU (1-rank RCCL group, forced bucketed all-reduce)
R=$GRAFT_REPO_ROOT
cd $R
T="timeout -k 10"
cd /tmp && export TMPDIR=/tmp
$T 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/r3s_dp -- python3 $R/tools/dp_timeline.py --steps 4 > $R/gpurun_out/r3s_dp.log 2>&1 || { tail -20 $R/gpurun_out/r3s_dp.log; exit 1; }
cd $R
t=$(find gpurun_out/r3s_dp -name '*kernel_trace.csv' | head -1); python3 tools/dp_timeline.py --summarize $t > gpurun_out/r3s_dp_timeline.txt 2>&1
head -40 gpurun_out/r3s_dp_timeline.txt
