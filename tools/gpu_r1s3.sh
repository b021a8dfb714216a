tools/gpurun_steps.sh \
 "500|pytest_gpu|python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread" \
 "200|smoke|python -c 'import __graft_entry__ as g; g.smoke()'" \
 "300|bench|python bench.py --steps 30 --warmup 5"
