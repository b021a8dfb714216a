# Round 3 step A: GPU tests of the cleaned-up local track + new GEMM / GO head kernels, headline bench,
# and the REFERENCE modules.py step on the same box (BASELINE cfg 2 shape)
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 300 python -u -m pytest tests/test_hip_gemm.py -x -q -s --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r3a_gemm_tests.log 2>&1 || { tail -60 gpurun_out/r3a_gemm_tests.log; exit 1; }
tail -3 gpurun_out/r3a_gemm_tests.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -s --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r3a_gpu_tests.log 2>&1 || { tail -60 gpurun_out/r3a_gpu_tests.log; exit 1; }
tail -3 gpurun_out/r3a_gpu_tests.log
timeout -k 10 300 python -u bench.py > gpurun_out/r3a_bench.json 2> gpurun_out/r3a_bench.err || exit 1
cat gpurun_out/r3a_bench.json
for b in 64 256; do
  timeout -k 10 400 python -u tools/ref_bench.py --batch $b --steps 10 --warmup 3 > gpurun_out/r3_ref_b$b.json 2> gpurun_out/r3_ref_b$b.err || exit 1
  cat gpurun_out/r3_ref_b$b.json
done
