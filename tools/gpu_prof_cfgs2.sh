# serial kernel stats (PBX_AUX_STREAM=0): cfg 4 (L=4096), cfg 5 (fine-tune) and paper semantics (L=512)
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
PBX_AUX_STREAM=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof2_c4 -- python3 $R/bench.py --steps 3 --warmup 2 --preset cfg4_long_l4096_dp8 > $R/gpurun_out/prof2_c4.log 2>&1 && \
PBX_AUX_STREAM=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof2_c5 -- python3 $R/bench.py --steps 3 --warmup 2 --mode finetune > $R/gpurun_out/prof2_c5.log 2>&1 && \
PBX_AUX_STREAM=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof2_pp -- python3 $R/bench.py --steps 3 --warmup 2 --semantics paper > $R/gpurun_out/prof2_pp.log 2>&1
echo rc=$?
