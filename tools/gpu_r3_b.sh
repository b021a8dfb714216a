# Round 3 step B: new-kernel GPU tests first (GEMM / GO head / local head), then the full GPU suite,
# the headline bench with and without the fused global-track backward on its aux stream, and the
# REFERENCE modules.py step on the same box.
R=$GRAFT_REPO_ROOT
cd $R
T="timeout -k 10"
$T 300 python -u -m pytest tests/test_hip_gemm.py tests/test_hip_heads.py -x -q -s --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r3b_new_tests.log 2>&1 || { tail -60 gpurun_out/r3b_new_tests.log; exit 1; }
tail -3 gpurun_out/r3b_new_tests.log
$T 900 python -u -m pytest tests -m gpu -x -q -s --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r3b_gpu_tests.log 2>&1 || { tail -60 gpurun_out/r3b_gpu_tests.log; exit 1; }
tail -3 gpurun_out/r3b_gpu_tests.log
for i in 1 2; do
  $T 300 python -u bench.py > gpurun_out/r3b_bench_$i.json 2> gpurun_out/r3b_bench_$i.err || exit 1
  PBX_GLOBAL_STREAM=1 $T 300 python -u bench.py > gpurun_out/r3b_bench_gs_$i.json 2> gpurun_out/r3b_bench_gs_$i.err || exit 1
  python3 -c "import json;a=json.load(open('gpurun_out/r3b_bench_$i.json'));b=json.load(open('gpurun_out/r3b_bench_gs_$i.json'));print('default',a['value'],a['ms_per_step'],'| global-stream',b['value'],b['ms_per_step'])"
done
for b in 64 256; do
  $T 400 python -u tools/ref_bench.py --batch $b --steps 10 --warmup 3 > gpurun_out/r3_ref_b$b.json 2> gpurun_out/r3_ref_b$b.err || exit 1
  cat gpurun_out/r3_ref_b$b.json
done
