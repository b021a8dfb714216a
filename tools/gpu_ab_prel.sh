cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_hip_local_track.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_local2.log 2>&1 || { tail -30 gpurun_out/t_local2.log; exit 1; }
tail -2 gpurun_out/t_local2.log
bash tools/ab_envs.sh 2 "PBX_PRE_L=store" "PBX_PRE_L=recompute" "PBX_PRE_L=store PBX_LN2_WGCU=2" "PBX_PRE_L=recompute PBX_LN2_WGCU=2"
