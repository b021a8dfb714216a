tools/gpurun_steps.sh \
 "200|kbench|python tools/kbench.py" \
 "300|pytest_hip|python -u -m pytest tests/test_hip_local_track.py tests/test_graph_step.py -x -q --timeout 120 --timeout-method thread" \
 "200|bench|python bench.py --steps 60 --warmup 5" \
 "200|bench2|python bench.py --steps 60 --warmup 5"
