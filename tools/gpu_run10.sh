tools/gpurun_steps.sh \
 "400|pytest_hip|python -m pytest tests/test_hip_local_track.py tests/test_graph_step.py -q -x" \
 "200|kbench_attn|python tools/kbench_attn.py" \
 "300|bench_hip|python bench.py --steps 30 --warmup 5"
