tools/gpurun_steps.sh \
 "400|pytest_hip|python -m pytest tests/test_hip_local_track.py -x -q -v" \
 "300|pytest_gpu_all|python -m pytest tests -m gpu -q"
