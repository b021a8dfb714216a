# GPU tests of the long-sequence changes, then the L=512 / 1024 / 4096 benches
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_hip_heads.py tests/test_hip_local_track.py tests/test_hip_global_track.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t_long.log 2>&1 || { tail -40 gpurun_out/t_long.log; exit 1; }
tail -2 gpurun_out/t_long.log
for cfg in cfg2_paper_l512 cfg3_paper_l1024_dp8 cfg4_long_l4096_dp8; do
  timeout -k 10 300 python -u bench.py --preset $cfg > gpurun_out/bl_$cfg.json 2> gpurun_out/bl_$cfg.err || { tail -5 gpurun_out/bl_$cfg.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/bl_$cfg.json'));print('$cfg', d['value'], d['ms_per_step'], d['config']['per_gpu_batch'])"
done
