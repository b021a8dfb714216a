tools/gpurun_steps.sh \
 "400|pytest_hip|python -m pytest tests/test_hip_local_track.py tests/test_graph_step.py -q -x" \
 "200|smoke|python -c 'import __graft_entry__ as g; g.smoke()'" \
 "300|bench_hip|python bench.py --steps 30 --warmup 5" \
 "400|prof_hip|cd /tmp && export TMPDIR=/tmp && rocprofv3 --kernel-trace --stats --output-format csv -d \$GRAFT_REPO_ROOT/gpurun_out/prof_hip5 -- python3 \$GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 3"
