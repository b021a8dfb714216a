tools/gpurun_steps.sh \
 "200|t|python -u -m pytest tests/test_hip_local_track.py -x -q --timeout 120 --timeout-method thread" \
 "100|ka|python tools/kbench_attn.py" \
 "100|b1|python bench.py --steps 60 --warmup 5"
