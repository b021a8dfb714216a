# v8 check: full GPU suite, smoke, headline bench x3, and the step's kernel list (serial profile)
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/v8_full_gpu_tests.log 2>&1 || { tail -40 gpurun_out/v8_full_gpu_tests.log; exit 1; }
tail -1 gpurun_out/v8_full_gpu_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/v8_smoke.log 2>&1 || { tail -20 gpurun_out/v8_smoke.log; exit 1; }
tail -1 gpurun_out/v8_smoke.log
for r in 1 2 3; do
  timeout -k 10 300 python -u bench.py > gpurun_out/v8_bench_l512_$r.json 2>/dev/null || exit 1
  echo "bench run $r: $(python3 -c "import json;d=json.load(open('gpurun_out/v8_bench_l512_$r.json'));print(d['value'], d['ms_per_step'])")"
done
bash tools/gpu_prof_serial.sh r2_v8b_serial || exit 1
f=$(find gpurun_out/r2_v8b_serial -name '*kernel_stats.csv' | head -1); python3 tools/profsum.py $f 8 40 > gpurun_out/r2_v8b_serial_summary.txt
head -3 gpurun_out/r2_v8b_serial_summary.txt
