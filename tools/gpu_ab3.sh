tools/gpurun_steps.sh \
 "200|pytest_graph|python -u -m pytest tests/test_graph_step.py tests/test_gpu_ddp_streams.py -x -q --timeout 120 --timeout-method thread" \
 "100|hp_glob|python bench.py --steps 60 --warmup 5" \
 "100|hp_noglob|PBX_GLOBAL_STREAM=0 python bench.py --steps 60 --warmup 5" \
 "100|nohp_noglob|PBX_PRIORITY_STREAM=0 PBX_GLOBAL_STREAM=0 python bench.py --steps 60 --warmup 5" \
 "100|hp_glob2|python bench.py --steps 60 --warmup 5" \
 "100|hp_noglob2|PBX_GLOBAL_STREAM=0 python bench.py --steps 60 --warmup 5" \
 "100|nohp_noglob2|PBX_PRIORITY_STREAM=0 PBX_GLOBAL_STREAM=0 python bench.py --steps 60 --warmup 5"
