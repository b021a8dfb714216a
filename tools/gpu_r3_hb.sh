R=$GRAFT_REPO_ROOT
cd $R
PBX_HB_PROFILE=1 timeout -k 10 300 python -u tools/host_breakdown.py --steps 20 > gpurun_out/r3hb_host_breakdown.txt 2>&1 || { tail -20 gpurun_out/r3hb_host_breakdown.txt; exit 1; }
cat gpurun_out/r3hb_host_breakdown.txt
