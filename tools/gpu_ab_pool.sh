# same-box A/B of the attention-pool forms (alternating runs)
tools/gpurun_steps.sh \
 "120|v2a|python bench.py --steps 30" \
 "120|v1a|PBX_ATTN_POOL=v1 python bench.py --steps 30" \
 "120|v2b|python bench.py --steps 30" \
 "120|v1b|PBX_ATTN_POOL=v1 python bench.py --steps 30" \
 "120|ft2|python bench.py --mode finetune --steps 30" \
 "120|ft1|PBX_ATTN_POOL=v1 python bench.py --mode finetune --steps 30"
