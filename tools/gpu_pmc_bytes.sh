# HBM bytes per kernel of the headline step (FETCH_SIZE / WRITE_SIZE, one derived counter per pass)
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
run() {
  d=$1; shift
  rm -rf $R/gpurun_out/$d
  timeout -s KILL 150 rocprofv3 --pmc "$@" --output-format csv -d $R/gpurun_out/$d -- python3 $R/bench.py --steps 2 --warmup 1 > $R/gpurun_out/$d.log 2>&1
}
run pbytesF FETCH_SIZE GRBM_GUI_ACTIVE && run pbytesW WRITE_SIZE GRBM_GUI_ACTIVE
echo rc=$?
