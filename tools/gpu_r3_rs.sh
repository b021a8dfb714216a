# Round 3 step RS: conv weight-gradient chunk count R sweep on the current step (same box, 2 rounds)
R_=$GRAFT_REPO_ROOT
cd $R_
T="timeout -k 10"
for i in 1 2; do
  for r in 56 48 40 64; do PBX_WGRAD_R=$r $T 300 python -u bench.py > gpurun_out/r3rs_bench_R${r}_$i.json 2> gpurun_out/r3rs_bench_R${r}_$i.err || exit 1; python3 -c "import json;d=json.load(open('gpurun_out/r3rs_bench_R${r}_$i.json'));print('R=$r',d['value'],d['ms_per_step'])"; done
done
# run-to-run spread of the default bench (50 timed steps after the change) on the same box
for i in 1 2 3; do $T 300 python -u bench.py > gpurun_out/r3rs_bench_default_$i.json 2> gpurun_out/r3rs_bench_default_$i.err || exit 1; python3 -c "import json;d=json.load(open('gpurun_out/r3rs_bench_default_$i.json'));print('default',d['value'],d['ms_per_step'],d['steps'])"; done
