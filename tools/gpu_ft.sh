tools/gpurun_steps.sh \
 "200|ft|python bench.py --mode finetune --steps 30 --warmup 5" \
 "200|b1|python bench.py --steps 60 --warmup 5" \
 "200|l1024|python bench.py --steps 30 --warmup 5 --preset cfg3_paper_l1024_dp8" \
 "200|l4096|python bench.py --steps 20 --warmup 3 --preset cfg4_long_l4096_dp8"
