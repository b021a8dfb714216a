# A/B: HIP hardware queues per process (default 4) for the multi-stream step
cd $GRAFT_REPO_ROOT
T="timeout -k 10"
O=gpurun_out/r3_hwq2
mkdir -p $O
for i in 1 2 3 4 5 6; do
for q in 8 4; do GPU_MAX_HW_QUEUES=$q $T 300 python -u bench.py > $O/bench_q${q}_$i.json 2> $O/bench_q${q}_$i.err || exit 1; python3 -c "import json;d=json.load(open('$O/bench_q${q}_$i.json'));print('hw_queues=$q',d['value'],d['ms_per_step'])"; done
done
