# LN1 backward fused into the conv data gradient: local-track + model GPU tests, then same-box step A/B
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_hip_local_track.py tests/test_determinism.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ln1f_tests.log 2>&1 || { tail -40 gpurun_out/ln1f_tests.log; exit 1; }
tail -1 gpurun_out/ln1f_tests.log
bash tools/ab_envs.sh 3 "PBX_LN1_FUSE=1" "PBX_LN1_FUSE=0"
