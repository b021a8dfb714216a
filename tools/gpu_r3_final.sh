# Round 3 final tree: full GPU suite, smoke, headline bench (x2) and the other BASELINE configurations
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out/r3_final4
O=gpurun_out/r3_final4
T="timeout -k 10"
PBX_LAUNCHER_REPORT=$O/launcher_coverage.txt $T 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
$T 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
for i in 1 2 3; do $T 300 python -u bench.py > $O/bench_l512_run$i.json 2> $O/bench_l512_run$i.err || exit 1; done
cat $O/bench_l512_run*.json
$T 300 python -u bench.py --semantics paper > $O/bench_paper.json 2> $O/bench_paper.err || exit 1
$T 300 python -u bench.py --preset cfg3_paper_l1024_dp8 > $O/bench_l1024.json 2> $O/bench_l1024.err || exit 1
$T 300 python -u bench.py --preset cfg4_long_l4096_dp8 > $O/bench_l4096.json 2> $O/bench_l4096.err || exit 1
$T 300 python -u bench.py --mode finetune > $O/bench_ft.json 2> $O/bench_ft.err || exit 1
for f in paper l1024 l4096 ft; do python3 -c "import json;d=json.load(open('$O/bench_$f.json'));print('$f', d['value'], d['ms_per_step'], d['config'].get('per_gpu_batch'))"; done
