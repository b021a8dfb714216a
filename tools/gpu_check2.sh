tools/gpurun_steps.sh \
 "400|pytest_gpu|python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
 "200|bench|python bench.py --steps 40 --warmup 5" \
 "200|kbench_attn|python tools/kbench_attn.py" \
 "200|kbench|python tools/kbench.py"
