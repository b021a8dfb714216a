#!/bin/bash
# One parameterised runner for every GPU-box task (replaces the one-off gpu_*.sh scripts of rounds 1-3).
#
#   tools/gpu.sh <task> [args...] [-- <task> [args...]]...
#
# Tasks (each GPU step runs under its own `timeout -k 10`; a fault, abort, segfault or time limit
# stops the whole script -- no further GPU step runs after it):
#   tests [pytest args]                  pytest -m gpu (one process, per-test thread timeout)
#   smoke                                __graft_entry__.smoke()
#   bench <tag> [bench.py args]          one bench run -> gpurun_out/<tag>.json
#   ab <tag> "<envA>" "<envB>" <rounds> [bench.py args]
#                                        same-box A/B of bench.py under two env settings, alternated
#   prof <tag> [bench.py args]           rocprofv3 kernel trace + stats of a short bench run,
#                                        summarised by tools/profsum.py / tools/critpath.py
#   pmc <tag> <counters> [bench.py args] one rocprofv3 --pmc pass (counters comma-separated, within
#                                        the per-block limits) over a short bench run
#   py <tag> <seconds> <script> [args]   any python script (a probe under tools/) with a time limit
#   profpy <tag> <seconds> <script> [args]  rocprofv3 kernel trace + stats of any python script
# Example:
#   gpurun --timeout 900 -- 'bash tools/gpu.sh tests -- bench r4_base --steps 50 -- prof r4_prof'
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
export TMPDIR=/tmp
T="timeout -k 10"

fatal() { local rc=$1; shift; echo "FATAL rc=$rc in $*; stopping" | tee -a gpurun_out/gpu.log; exit "$rc"; }
ok_or_stop() {   # pytest failures (rc 1) are results; anything else ends the script
  local rc=$1; shift
  if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then fatal "$rc" "$@"; fi
}
summ() { python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[2],d['value'],d['ms_per_step'],d['config'].get('hip_graph'))" "$@"; }

run_task() {
  local task=$1; shift
  echo "=== $task $* ($(date +%T))" | tee -a gpurun_out/gpu.log
  case "$task" in
    tests)
      $T 1500 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread "$@" \
        > gpurun_out/gpu_tests.log 2>&1
      local rc=$?; tail -3 gpurun_out/gpu_tests.log; ok_or_stop $rc tests ;;
    smoke)
      $T 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || fatal $? smoke
      tail -1 gpurun_out/smoke.log ;;
    bench)
      local tag=$1; shift
      $T 400 python -u bench.py "$@" > gpurun_out/$tag.json 2> gpurun_out/$tag.err || fatal $? "bench $tag"
      summ gpurun_out/$tag.json "$tag" ;;
    ab)
      local tag=$1 A=$2 B=$3 rounds=$4; shift 4
      for i in $(seq 1 "$rounds"); do
        for k in A B; do
          local envs; envs=$([ $k = A ] && echo "$A" || echo "$B")
          env $envs $T 400 python -u bench.py "$@" > gpurun_out/${tag}_${k}_$i.json 2> gpurun_out/${tag}_${k}_$i.err \
            || fatal $? "ab $tag $k"
          summ gpurun_out/${tag}_${k}_$i.json "$k[$envs]"
        done
      done ;;
    prof)
      local tag=$1; shift
      rm -rf gpurun_out/$tag
      $T 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$tag -o run -- python3 -u bench.py --steps 10 --warmup 3 "$@" \
        > gpurun_out/$tag.log 2>&1 || fatal $? "prof $tag"
      local st tr
      st=$(find gpurun_out/$tag -name '*kernel_stats.csv' | head -1)
      tr=$(find gpurun_out/$tag -name '*kernel_trace.csv' | head -1)
      python3 tools/profsum.py "$st" 13 40 > gpurun_out/${tag}_summary.txt 2>&1 || true
      python3 tools/critpath.py "$tr" > gpurun_out/${tag}_critpath.txt 2>&1 || true
      head -25 gpurun_out/${tag}_summary.txt ;;
    profpy)
      local tag=$1 secs=$2; shift 2
      rm -rf gpurun_out/$tag
      $T "$secs" rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$tag -o run -- python3 -u "$@" \
        > gpurun_out/$tag.log 2>&1 || fatal $? "profpy $tag"
      tail -3 gpurun_out/$tag.log ;;
    pmc)
      local tag=$1 ctr=$2; shift 2
      rm -rf gpurun_out/$tag
      timeout -s KILL 300 rocprofv3 --kernel-trace --output-format csv --pmc ${ctr//,/ } -d gpurun_out/$tag -o run -- \
        python3 -u bench.py --steps 3 --warmup 2 "$@" > gpurun_out/$tag.log 2>&1 || fatal $? "pmc $tag"
      echo "pmc $tag done" ;;
    py)
      local tag=$1 secs=$2; shift 2
      $T "$secs" python -u "$@" > gpurun_out/$tag.log 2>&1 || fatal $? "py $tag"
      tail -20 gpurun_out/$tag.log ;;
    *) echo "unknown task $task"; exit 2 ;;
  esac
}

args=()
for a in "$@" "--"; do
  if [ "$a" = "--" ]; then
    [ ${#args[@]} -gt 0 ] && run_task "${args[@]}"
    args=()
  else
    args+=("$a")
  fi
done
exit 0
