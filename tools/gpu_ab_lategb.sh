# late-gb GPU tests, pool microbench (current vs no-GELU ablation), then same-box A/B of the step
cd $GRAFT_REPO_ROOT
timeout -k 10 60 ./tools/ubench/gelu_ubench > gpurun_out/gelu_ub.log 2>&1 && cat gpurun_out/gelu_ub.log
timeout -k 10 400 python -u -m pytest tests/test_hip_local_track.py tests/test_graph_step.py -x -q --timeout 150 --timeout-method thread > gpurun_out/t_late.log 2>&1 || { tail -40 gpurun_out/t_late.log; exit 1; }
tail -2 gpurun_out/t_late.log
bash tools/gpu_poolbench.sh || exit 1
bash tools/ab_envs.sh 2 "PBX_LATE_GB=0" "PBX_LATE_GB=1"
