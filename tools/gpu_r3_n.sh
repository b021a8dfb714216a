# Round 3 step N: sparse GO input layer (csrc/annot.hip) - numerics vs fp32, same-box bench A/B, trace
R=$GRAFT_REPO_ROOT
cd $R
T="timeout -k 10"
$T 600 python -u -m pytest tests/test_hip_input_layer.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r3n_tests.log 2>&1 || { grep -E "Error|assert|FAIL|failed" gpurun_out/r3n_tests.log | tail -30; exit 1; }
tail -1 gpurun_out/r3n_tests.log
for i in 1 2 3; do
  for v in 1 0; do PBX_ANN_SPARSE=$v $T 300 python -u bench.py > gpurun_out/r3n_bench_s${v}_$i.json 2> gpurun_out/r3n_bench_s${v}_$i.err || exit 1; python3 -c "import json;d=json.load(open('gpurun_out/r3n_bench_s${v}_$i.json'));print('ann_sparse=$v',d['value'],d['ms_per_step'])"; done
done
cd /tmp && export TMPDIR=/tmp
$T 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r3n_conc -- python3 $R/bench.py --steps 5 --warmup 3 > $R/gpurun_out/r3n_conc.log 2>&1 || exit 1
cd $R
t=$(find gpurun_out/r3n_conc -name '*kernel_trace.csv' | head -1); python3 tools/critpath.py $t 2 > gpurun_out/r3n_critpath.txt
grep -E "ann_|span|queue" gpurun_out/r3n_critpath.txt | head -20
