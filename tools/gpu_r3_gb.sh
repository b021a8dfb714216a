# Round 3 final tree: column-split global-track backward (PBX_GLOB3_BWD=1) vs the one-launch backward, same box, 3 rounds
R=$GRAFT_REPO_ROOT
cd $R
T="timeout -k 10"
for i in 1 2 3; do
  for v in 1 0; do PBX_GLOB3_BWD=$v $T 300 python -u bench.py > gpurun_out/r3gb_bench_b${v}_$i.json 2> gpurun_out/r3gb_bench_b${v}_$i.err || exit 1; python3 -c "import json;d=json.load(open('gpurun_out/r3gb_bench_b${v}_$i.json'));print('glob3_bwd=$v',d['value'],d['ms_per_step'])"; done
done
