# Round 3 step S: data-parallel overlap timeline on one GPU (1-rank RCCL group, forced bucketed all-reduce, HIP events)
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 300 python3 tools/dp_timeline.py --steps 6 > gpurun_out/r3s_dp_timeline.txt 2>&1 || { tail -20 gpurun_out/r3s_dp_timeline.txt; exit 1; }
cat gpurun_out/r3s_dp_timeline.txt
