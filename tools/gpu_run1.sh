tools/gpurun_steps.sh \
 "300|pytest_gpu|python -m pytest tests -m gpu -x -q" \
 "300|bench_torch|python bench.py --impl torch --steps 10 --warmup 3" \
 "300|bench_faithful|python bench.py --impl faithful --steps 5 --warmup 2 --batch 64" \
 "400|prof_torch|cd /tmp && export TMPDIR=/tmp && rocprofv3 --kernel-trace --stats --output-format csv -d \$GRAFT_REPO_ROOT/gpurun_out/prof_torch -- python3 \$GRAFT_REPO_ROOT/bench.py --impl torch --steps 3 --warmup 2"
