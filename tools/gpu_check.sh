# GPU correctness + headline bench (each step time-limited; a fatal step stops the script)
tools/gpurun_steps.sh \
 "400|pytest_gpu|python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
 "200|bench|python bench.py --steps 30 --warmup 5" \
 "200|bench_v1|PBX_CONV=v1 python bench.py --steps 30 --warmup 5"
