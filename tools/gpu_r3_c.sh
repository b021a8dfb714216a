# Round 3 step C: new tests (determinism, multi-length), serial + concurrent kernel traces of the
# headline step, the deterministic-mode step cost, and the REFERENCE modules.py step (snapshot of the
# read-only reference file staged into .refsnap/ by the caller; never committed).
R=$GRAFT_REPO_ROOT
cd $R
T="timeout -k 10"
$T 400 python -u -m pytest tests/test_determinism.py tests/test_multilength.py -x -q -s --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r3c_tests.log 2>&1 || { tail -40 gpurun_out/r3c_tests.log; exit 1; }
grep -E "max \||passed|failed" gpurun_out/r3c_tests.log | tail -5
bash $R/tools/gpu_prof_serial.sh r3c_serial || exit 1
f=$(find gpurun_out/r3c_serial -name '*kernel_stats.csv' | head -1); python3 tools/profsum.py $f 8 40 > gpurun_out/r3c_serial_summary.txt
head -30 gpurun_out/r3c_serial_summary.txt
cd /tmp && export TMPDIR=/tmp
$T 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r3c_conc -- python3 $R/bench.py --steps 5 --warmup 3 > $R/gpurun_out/r3c_conc.log 2>&1 || exit 1
cd $R
t=$(find gpurun_out/r3c_conc -name '*kernel_trace.csv' | head -1); python3 tools/stepspan.py $t 4 > gpurun_out/r3c_conc_steps.txt
head -40 gpurun_out/r3c_conc_steps.txt
$T 300 python -u bench.py > gpurun_out/r3c_bench.json 2> gpurun_out/r3c_bench.err || exit 1
PBX_DETERMINISTIC=1 $T 300 python -u bench.py > gpurun_out/r3c_bench_det.json 2> gpurun_out/r3c_bench_det.err || exit 1
python3 -c "import json;a=json.load(open('gpurun_out/r3c_bench.json'));b=json.load(open('gpurun_out/r3c_bench_det.json'));print('default',a['value'],a['ms_per_step'],'| deterministic',b['value'],b['ms_per_step'])"
for b in 64 256; do
  PBX_REFERENCE_DIR=$R/.refsnap $T 400 python -u tools/ref_bench.py --batch $b --steps 10 --warmup 3 > gpurun_out/r3_ref_b$b.json 2> gpurun_out/r3_ref_b$b.err || exit 1
  cat gpurun_out/r3_ref_b$b.json
done
