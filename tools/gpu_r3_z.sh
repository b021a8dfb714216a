# Round 3 step Z: run-to-run variance on one box: eager vs hipGraph step, host issue time, GPU clocks
R=$GRAFT_REPO_ROOT
cd $R
T="timeout -k 10"
cat /proc/loadavg > gpurun_out/r3z_env.txt; nproc >> gpurun_out/r3z_env.txt
(rocm-smi --showclocks --showtemp --showpower 2>&1 | head -40) >> gpurun_out/r3z_env.txt || true
for i in 1 2 3; do
  $T 300 python -u bench.py --graph off > gpurun_out/r3z_bench_eager_$i.json 2> gpurun_out/r3z_bench_eager_$i.err || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/r3z_bench_eager_$i.json'));print('eager',d['value'],d['ms_per_step'])"
  $T 300 python -u bench.py --graph on > gpurun_out/r3z_bench_graph_$i.json 2> gpurun_out/r3z_bench_graph_$i.err || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/r3z_bench_graph_$i.json'));print('graph',d['value'],d['ms_per_step'],d['config']['hip_graph'])"
  $T 300 python -u tools/cpu_overhead.py --steps 30 2>&1 | grep issue
  cat /proc/loadavg
done
(rocm-smi --showclocks --showtemp --showpower 2>&1 | head -40) >> gpurun_out/r3z_env.txt || true
