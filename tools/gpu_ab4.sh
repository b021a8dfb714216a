tools/gpurun_steps.sh \
 "200|gt|python -u -m pytest tests/test_hip_global_track.py -x -q --timeout 120 --timeout-method thread" \
 "100|fused|python bench.py --steps 60 --warmup 5" \
 "100|lib|PBX_GLOBAL_FUSED=0 python bench.py --steps 60 --warmup 5" \
 "100|fused2|python bench.py --steps 60 --warmup 5" \
 "100|lib2|PBX_GLOBAL_FUSED=0 python bench.py --steps 60 --warmup 5" \
 "300|prof|bash tools/gpu_prof.sh prof_g2"
