tools/gpurun_steps.sh \
 "400|pytest_hip|python -m pytest tests/test_hip_local_track.py tests/test_graph_step.py -q -x" \
 "200|kbench_attn|python tools/kbench_attn.py" \
 "300|kbench|python tools/kbench.py" \
 "300|attn_dbg|bash tools/gpu_attn_dbg.sh" \
 "300|bench_hip|python bench.py --steps 30 --warmup 5" \
 "400|prof_hip|cd /tmp && export TMPDIR=/tmp && rocprofv3 --kernel-trace --stats --output-format csv -d \$GRAFT_REPO_ROOT/gpurun_out/prof_hip6 -- python3 \$GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 3"
