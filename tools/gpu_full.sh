# Round-end style check: full GPU test suite, smoke, headline bench and the other BASELINE configs.
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/full_gpu_tests.log 2>&1 || { tail -40 gpurun_out/full_gpu_tests.log; exit 1; }
tail -3 gpurun_out/full_gpu_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/full_smoke.log 2>&1 || { tail -20 gpurun_out/full_smoke.log; exit 1; }
timeout -k 10 300 python -u bench.py > gpurun_out/full_bench_l512.json 2> gpurun_out/full_bench_l512.err || exit 1
cat gpurun_out/full_bench_l512.json
timeout -k 10 300 python -u bench.py --semantics paper > gpurun_out/full_bench_paper.json 2> gpurun_out/full_bench_paper.err || exit 1
timeout -k 10 300 python -u bench.py --preset cfg3_paper_l1024_dp8 > gpurun_out/full_bench_l1024.json 2> gpurun_out/full_bench_l1024.err || exit 1
timeout -k 10 300 python -u bench.py --preset cfg4_long_l4096_dp8 > gpurun_out/full_bench_l4096.json 2> gpurun_out/full_bench_l4096.err || exit 1
timeout -k 10 300 python -u bench.py --mode finetune > gpurun_out/full_bench_ft.json 2> gpurun_out/full_bench_ft.err || exit 1
for f in paper l1024 l4096 ft; do python3 -c "import json;d=json.load(open('gpurun_out/full_bench_$f.json'));print('$f', d['value'], d['ms_per_step'], d['config'].get('per_gpu_batch'))"; done
