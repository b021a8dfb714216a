tools/gpurun_steps.sh \
 "200|c2|python bench.py --steps 30 --warmup 5" \
 "200|c2b|python bench.py --steps 30 --warmup 5" \
 "200|c3|python bench.py --steps 20 --warmup 5 --preset cfg3_paper_l1024_dp8" \
 "200|c4|python bench.py --steps 10 --warmup 3 --preset cfg4_long_l4096_dp8" \
 "200|c5|python bench.py --mode finetune --steps 30 --warmup 5" \
 "300|prof|bash tools/gpu_prof.sh prof_b512"
