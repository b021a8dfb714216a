# Round 3: long headline runs (200 timed steps) + host issue time, to document the run-to-run spread
R=$GRAFT_REPO_ROOT
cd $R
T="timeout -k 10"
cat /proc/loadavg
for i in 1 2 3; do $T 300 python -u bench.py --steps 200 --warmup 20 > gpurun_out/r3long_bench_$i.json 2> gpurun_out/r3long_bench_$i.err || exit 1; python3 -c "import json;d=json.load(open('gpurun_out/r3long_bench_$i.json'));print('200-step',d['value'],d['ms_per_step'])"; $T 300 python -u tools/cpu_overhead.py --steps 30 2>&1 | grep issue; cat /proc/loadavg; done
