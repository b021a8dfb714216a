cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_finetune.py tests/test_hip_local_track.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/t_ft.log 2>&1 || { tail -40 gpurun_out/t_ft.log; exit 1; }
tail -2 gpurun_out/t_ft.log
timeout -k 10 300 python -u bench.py --mode finetune > gpurun_out/bf_c5.json 2> gpurun_out/bf_c5.err || { tail -5 gpurun_out/bf_c5.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/bf_c5.json'));print('cfg5', d['value'], d['ms_per_step'])"
for cfg in cfg4_long_l4096_dp8 cfg2_paper_l512; do
  timeout -k 10 300 python -u bench.py --preset $cfg > gpurun_out/bl_$cfg.json 2> gpurun_out/bl_$cfg.err || { tail -5 gpurun_out/bl_$cfg.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/bl_$cfg.json'));print('$cfg', d['value'], d['ms_per_step'], d['config']['per_gpu_batch'])"
done
