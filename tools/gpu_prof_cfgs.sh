# serial kernel stats (PBX_AUX_STREAM=0) of the L=4096 (cfg 4) and L=1024 (cfg 3) steps
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
PBX_AUX_STREAM=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_c4 -- python3 $R/bench.py --steps 3 --warmup 2 --preset cfg4_long_l4096_dp8 > $R/gpurun_out/prof_c4.log 2>&1 && \
PBX_AUX_STREAM=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_c3 -- python3 $R/bench.py --steps 3 --warmup 2 --preset cfg3_paper_l1024_dp8 > $R/gpurun_out/prof_c3.log 2>&1
echo rc=$?
