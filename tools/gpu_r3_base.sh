# Round 3: GPU tests (local track + full model), headline bench (x2), and the REFERENCE modules.py step
# on the same box (BASELINE cfg 2 shape)
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -s --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r3_gpu_tests.log 2>&1 || { tail -60 gpurun_out/r3_gpu_tests.log; exit 1; }
tail -3 gpurun_out/r3_gpu_tests.log
for i in 1 2; do
  timeout -k 10 300 python -u bench.py > gpurun_out/r3_base_bench_$i.json 2> gpurun_out/r3_base_bench_$i.err || exit 1
  cat gpurun_out/r3_base_bench_$i.json
done
for b in 64 256; do
  timeout -k 10 400 python -u tools/ref_bench.py --batch $b --steps 10 --warmup 3 > gpurun_out/r3_ref_b$b.json 2> gpurun_out/r3_ref_b$b.err || exit 1
  cat gpurun_out/r3_ref_b$b.json
done
