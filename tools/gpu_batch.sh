tools/gpurun_steps.sh \
 "200|b256|python bench.py --steps 30 --warmup 5" \
 "200|b512|python bench.py --steps 30 --warmup 5 --batch 512" \
 "200|b768|python bench.py --steps 20 --warmup 5 --batch 768" \
 "200|b1024|python bench.py --steps 20 --warmup 5 --batch 1024"
