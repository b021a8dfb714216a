# conv kernel change check: standalone timing + cross-check, then the local-track numerics tests
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 120 python -u tools/ubench/convbench.py --tag new > gpurun_out/convab.log 2>&1 || { cat gpurun_out/convab.log; exit 1; }
timeout -k 10 300 python -u -m pytest tests/test_hip_local_track.py tests/test_hip_paper_local.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/conv_tests.log 2>&1 || { tail -30 gpurun_out/conv_tests.log; exit 1; }
tail -3 gpurun_out/conv_tests.log
