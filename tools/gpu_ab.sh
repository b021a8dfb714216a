tools/gpurun_steps.sh \
 "100|e40|PBX_WGRAD_R=40 python bench.py --steps 40 --warmup 5 --graph off" \
 "100|e48|PBX_WGRAD_R=48 python bench.py --steps 40 --warmup 5 --graph off" \
 "100|e56|PBX_WGRAD_R=56 python bench.py --steps 40 --warmup 5 --graph off" \
 "100|e40b|PBX_WGRAD_R=40 python bench.py --steps 40 --warmup 5 --graph off" \
 "100|e48b|PBX_WGRAD_R=48 python bench.py --steps 40 --warmup 5 --graph off" \
 "100|e56b|PBX_WGRAD_R=56 python bench.py --steps 40 --warmup 5 --graph off" \
 "100|g48|PBX_WGRAD_R=48 python bench.py --steps 40 --warmup 5 --graph on"
