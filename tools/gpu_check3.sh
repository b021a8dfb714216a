tools/gpurun_steps.sh \
 "400|pytest_gpu|python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
 "200|bench|python bench.py --steps 60 --warmup 5" \
 "200|bench_noglob|PBX_GLOBAL_STREAM=0 python bench.py --steps 60 --warmup 5" \
 "200|bench2|python bench.py --steps 60 --warmup 5"
