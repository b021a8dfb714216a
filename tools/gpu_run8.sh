tools/gpurun_steps.sh \
 "500|pytest_gpu|python -m pytest tests -m gpu -q" \
 "300|bench_hip|python bench.py --steps 30 --warmup 5" \
 "400|prof_hip|cd /tmp && export TMPDIR=/tmp && rocprofv3 --kernel-trace --stats --output-format csv -d \$GRAFT_REPO_ROOT/gpurun_out/prof_hip4 -- python3 \$GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 3"
