tools/gpurun_steps.sh \
 "100|a1|python bench.py --steps 60 --warmup 5" \
 "100|a2|python bench.py --steps 60 --warmup 5" \
 "100|a3|python bench.py --steps 60 --warmup 5" \
 "100|a4|python bench.py --steps 60 --warmup 5" \
 "100|n1|PBX_AUX_STREAM=0 python bench.py --steps 60 --warmup 5" \
 "100|n2|PBX_AUX_STREAM=0 python bench.py --steps 60 --warmup 5" \
 "100|n3|PBX_AUX_STREAM=0 python bench.py --steps 60 --warmup 5"
