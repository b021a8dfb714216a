tools/gpurun_steps.sh \
 "300|kbench|python tools/kbench.py" \
 "300|bench_hip|python bench.py --steps 30 --warmup 5"
