# Round 3 step R: paper-semantics weight gradients on the in-tree split-K GEMM (was chunked library bmm) - tests, same-box A/B, kernel summary
R=$GRAFT_REPO_ROOT
cd $R
T="timeout -k 10"
$T 600 python -u -m pytest tests/test_hip_paper_local.py tests/test_hip_paper_attention.py tests/test_hip_input_layer.py -x -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r3r_tests.log 2>&1 || { grep -E "Error|assert|FAIL|failed" gpurun_out/r3r_tests.log | tail -30; exit 1; }
tail -1 gpurun_out/r3r_tests.log
for i in 1 2; do
  for v in gemm bmm; do PBX_PAPER_WGRAD=$v $T 300 python -u bench.py --semantics paper > gpurun_out/r3r_bench_paper_${v}_$i.json 2> gpurun_out/r3r_bench_paper_${v}_$i.err || exit 1; python3 -c "import json;d=json.load(open('gpurun_out/r3r_bench_paper_${v}_$i.json'));print('paper wgrad=$v',d['value'],d['ms_per_step'])"; done
done
cd /tmp && export TMPDIR=/tmp
$T 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r3r_paper -- python3 $R/bench.py --semantics paper --steps 5 --warmup 3 > $R/gpurun_out/r3r_paper_prof.log 2>&1 || exit 1
cd $R
s=$(find gpurun_out/r3r_paper -name '*kernel_stats.csv' | head -1); python3 tools/profsum.py $s 8 > gpurun_out/r3r_paper_kernel_summary.txt 2>&1 || true
head -16 gpurun_out/r3r_paper_kernel_summary.txt
