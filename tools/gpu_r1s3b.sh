tools/gpurun_steps.sh \
 "200|bench_eager|python bench.py --steps 20 --warmup 5 --graph off" \
 "200|bench_l1024|python bench.py --steps 20 --warmup 3 --preset cfg3_paper_l1024_dp8" \
 "300|bench_l4096|python bench.py --steps 10 --warmup 3 --preset cfg4_long_l4096_dp8" \
 "400|prof_hip|cd /tmp && export TMPDIR=/tmp && rocprofv3 --kernel-trace --stats --output-format csv -d \$GRAFT_REPO_ROOT/gpurun_out/prof_s3 -- python3 \$GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 3"
