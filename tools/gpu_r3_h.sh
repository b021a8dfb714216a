# Round 3 step H2: host-side cost of the eager step: issue time, cProfile, HIP API trace summary
R=$GRAFT_REPO_ROOT
cd $R
T="timeout -k 10"
cat /proc/loadavg
$T 300 python -u tools/cpu_overhead.py --steps 30 2>&1 | grep issue
$T 300 python -u bench.py > gpurun_out/r3h2_bench.json 2> gpurun_out/r3h2_bench.err || exit 1
python3 -c "import json;d=json.load(open('gpurun_out/r3h2_bench.json'));print('bench',d['value'],d['ms_per_step'])"
PBX_CPROFILE=1 $T 300 python -u tools/cpu_overhead.py --steps 10 > gpurun_out/r3h2_cprofile.txt 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
$T 300 rocprofv3 --hip-trace --stats --output-format csv -d $R/gpurun_out/r3h2_hip -- python3 $R/bench.py --steps 10 --warmup 3 > $R/gpurun_out/r3h2_hip.log 2>&1 || exit 1
cd $R
f=$(find gpurun_out/r3h2_hip -name '*hip_api_stats.csv' | head -1); head -25 $f > gpurun_out/r3h2_hip_api_stats.txt; cat gpurun_out/r3h2_hip_api_stats.txt | cut -c1-160
