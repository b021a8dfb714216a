#!/bin/bash
# Same-box A/B of an older checkout (a git worktree with its own built libraries, e.g. _r5) against this
# tree, each at its own default bench config, runs alternated:
#   gpurun -- 'bash tools/ab_tree.sh _r5 3 --steps 30 --warmup 5'
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
old=$1 rounds=$2; shift 2
for i in $(seq 1 "$rounds"); do
  (cd "$old" && timeout -k 10 400 python -u bench.py "$@") > gpurun_out/abtree_old_$i.json 2> gpurun_out/abtree_old_$i.err || exit $?
  timeout -k 10 400 python -u bench.py "$@" > gpurun_out/abtree_new_$i.json 2> gpurun_out/abtree_new_$i.err || exit $?
  for k in old new; do
    python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[2],d['value'],d['ms_per_step'],d['config']['per_gpu_batch'])" gpurun_out/abtree_${k}_$i.json "$k$i"
  done
done
