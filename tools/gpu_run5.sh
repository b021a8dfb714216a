tools/gpurun_steps.sh \
 "200|gemm_probe|python tools/gemm_probe.py" \
 "400|pytest_hip|python -m pytest tests/test_hip_local_track.py -x -q" \
 "300|bench_hip|python bench.py --steps 20 --warmup 5"
