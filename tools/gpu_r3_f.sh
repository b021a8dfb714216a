# Round 3 step F: LayerNorm-2 split out of the pool forward (PBX_POOL_PRENORM) - numerics, kernel time, step A/B
R=$GRAFT_REPO_ROOT
cd $R
T="timeout -k 10"
$T 400 python -u -m pytest tests/test_hip_local_track.py tests/test_determinism.py tests/test_multilength.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r3f_tests.log 2>&1 || { tail -40 gpurun_out/r3f_tests.log; exit 1; }
tail -2 gpurun_out/r3f_tests.log
for pre in 0 1; do $T 60 python -u tools/ubench/poolstamps.py tools/ubench/abl/libpbx_st.so $pre > gpurun_out/r3f_poolstamps_$pre.txt 2>&1 || exit 1; sed -n 2p gpurun_out/r3f_poolstamps_$pre.txt; done
for i in 1 2; do
for pre in 0 1; do PBX_POOL_PRENORM=$pre $T 300 python -u bench.py > gpurun_out/r3f_bench_pre${pre}_$i.json 2> gpurun_out/r3f_bench_pre${pre}_$i.err || exit 1; python3 -c "import json;d=json.load(open('gpurun_out/r3f_bench_pre${pre}_$i.json'));print('prenorm=$pre',d['value'],d['ms_per_step'])"; done
done
