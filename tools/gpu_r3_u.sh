# Round 3 step U: observed gradient errors of the fused model vs fp32 torch (to size the test tolerances)
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 300 python -u -m pytest "tests/test_hip_local_track.py::test_full_model_loss_and_grads_vs_torch" "tests/test_hip_local_track.py::test_arena_direct_grads_match_autograd_path" -x -q -s --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r3u_grad_errors.log 2>&1 || { tail -30 gpurun_out/r3u_grad_errors.log; exit 1; }
tail -1 gpurun_out/r3u_grad_errors.log
