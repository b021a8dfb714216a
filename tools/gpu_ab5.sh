tools/gpurun_steps.sh \
 "400|pytest_gpu|python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
 "100|b1|python bench.py --steps 60 --warmup 5" \
 "100|b2|python bench.py --steps 60 --warmup 5" \
 "300|prof|bash tools/gpu_prof.sh prof_g3"
