cd /tmp && export TMPDIR=/tmp && timeout 120 rocprofv3 --list-avail > $GRAFT_REPO_ROOT/gpurun_out/counters.txt 2>&1; echo rc=$?
