# rocprofv3 kernel stats of the paper-semantics step with every backward kernel on the main stream;
# $1 = output dir name under gpurun_out/
cd /tmp && export TMPDIR=/tmp && export PBX_AUX_STREAM=0
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/$1 -- python3 $GRAFT_REPO_ROOT/bench.py --semantics paper --steps 5 --warmup 3 > $GRAFT_REPO_ROOT/gpurun_out/$1.log 2>&1
