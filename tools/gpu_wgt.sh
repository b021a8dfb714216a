cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
rm -rf $R/gpurun_out/wgT
timeout -s KILL 90 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/wgT -- python3 $R/tools/wgbench.py > $R/gpurun_out/wgT.log 2>&1
