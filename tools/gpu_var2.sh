tools/gpurun_steps.sh \
 "100|s1|python tools/steptimes.py 80" \
 "100|s2|python tools/steptimes.py 80" \
 "100|s3|PBX_AUX_STREAM=0 python tools/steptimes.py 80" \
 "100|b1|python bench.py --steps 60 --warmup 5" \
 "100|b2|python bench.py --steps 60 --warmup 5" \
 "100|b3|python bench.py --steps 60 --warmup 5"
