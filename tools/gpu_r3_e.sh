# Round 3 step E: host issue time vs GPU time of the eager step; eager vs hipGraph bench on one box.
R=$GRAFT_REPO_ROOT
cd $R
T="timeout -k 10"
$T 300 python -u tools/cpu_overhead.py > gpurun_out/r3e_cpu_overhead.txt 2>&1 || { cat gpurun_out/r3e_cpu_overhead.txt; exit 1; }
cat gpurun_out/r3e_cpu_overhead.txt
$T 300 python -u bench.py > gpurun_out/r3e_bench.json 2> gpurun_out/r3e_bench.err || exit 1
PBX_GRAPH=1 $T 300 python -u bench.py > gpurun_out/r3e_bench_graph.json 2> gpurun_out/r3e_bench_graph.err || { tail -5 gpurun_out/r3e_bench_graph.err; exit 1; }
$T 300 python -u bench.py > gpurun_out/r3e_bench2.json 2> gpurun_out/r3e_bench2.err || exit 1
PBX_GRAPH=1 $T 300 python -u bench.py > gpurun_out/r3e_bench_graph2.json 2> gpurun_out/r3e_bench_graph2.err || exit 1
for f in r3e_bench r3e_bench_graph r3e_bench2 r3e_bench_graph2; do python3 -c "import json;d=json.load(open('gpurun_out/$f.json'));print('$f',d['value'],d['ms_per_step'],d['config']['hip_graph'])"; done
