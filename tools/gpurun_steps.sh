#!/bin/bash
# Run GPU steps in sequence on the gpurun box; each step has its own time limit.
# A step that exits 0 or 1 (e.g. a pytest failure) lets the next one run; a fault,
# abort, segfault, or timeout (any other code) ends the script there.
# usage: tools/gpurun_steps.sh "<seconds>|<name>|<command>" ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for spec in "$@"; do
  secs="${spec%%|*}"; rest="${spec#*|}"; name="${rest%%|*}"; cmd="${rest#*|}"
  echo "=== [$name] ($secs s): $cmd" | tee -a gpurun_out/steps.log
  start=$(date +%s)
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "=== [$name] rc=$rc in $(( $(date +%s) - start ))s" | tee -a gpurun_out/steps.log
  tail -5 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
    echo "fatal rc=$rc in step $name; stopping" | tee -a gpurun_out/steps.log
    exit $rc
  fi
done
exit 0
