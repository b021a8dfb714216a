tools/gpurun_steps.sh \
 "200|pytest_graph|python -u -m pytest tests/test_graph_step.py -x -q --timeout 120 --timeout-method thread" \
 "200|b_eager_aux|python bench.py --steps 30 --warmup 5 --graph off" \
 "200|b_eager_noaux|PBX_AUX_STREAM=0 python bench.py --steps 30 --warmup 5 --graph off" \
 "200|b_graph_noaux|PBX_AUX_STREAM=0 python bench.py --steps 30 --warmup 5" \
 "300|prof_aux|bash tools/gpu_prof.sh prof_aux"
