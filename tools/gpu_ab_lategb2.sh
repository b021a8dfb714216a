cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_ddp_streams.py -x -q --timeout 150 --timeout-method thread > gpurun_out/t_ddp.log 2>&1 || { tail -30 gpurun_out/t_ddp.log; exit 1; }
tail -1 gpurun_out/t_ddp.log
bash tools/ab_envs.sh 2 "PBX_LATE_GB=0" "PBX_LATE_GB=1" "PBX_LATE_GB=1 PBX_GFWD_PRIO=0"
