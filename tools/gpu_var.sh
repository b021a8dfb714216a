tools/gpurun_steps.sh \
 "100|v1|python bench.py --steps 100 --warmup 10" \
 "100|v2|python bench.py --steps 100 --warmup 10" \
 "100|v3|python bench.py --steps 100 --warmup 10" \
 "100|n1|PBX_AUX_STREAM=0 python bench.py --steps 100 --warmup 10" \
 "100|n2|PBX_AUX_STREAM=0 python bench.py --steps 100 --warmup 10" \
 "100|v4|python bench.py --steps 20 --warmup 5"
