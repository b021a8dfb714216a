tools/gpurun_steps.sh \
 "400|pytest_hip|python -m pytest tests/test_hip_local_track.py -x -q" \
 "300|bench_hip|python bench.py --steps 20 --warmup 5" \
 "400|prof_hip|cd /tmp && export TMPDIR=/tmp && rocprofv3 --kernel-trace --stats --output-format csv -d \$GRAFT_REPO_ROOT/gpurun_out/prof_hip2 -- python3 \$GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 3"
