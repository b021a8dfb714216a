# GPU correctness + headline bench (each step time-limited; a fatal step stops the script)
tools/gpurun_steps.sh \
 "400|pytest_gpu|python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
 "200|smoke|python -c 'import __graft_entry__ as g; g.smoke()'" \
 "200|bench|python bench.py --steps 40 --warmup 5" \
 "200|bench2|python bench.py --steps 40 --warmup 5"
