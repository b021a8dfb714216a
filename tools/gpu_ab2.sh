tools/gpurun_steps.sh \
 "200|bench|python bench.py --steps 40 --warmup 5" \
 "200|kbench_attn|python tools/kbench_attn.py" \
 "200|kbench|python tools/kbench.py" \
 "200|bench2|python bench.py --steps 40 --warmup 5"
