#!/bin/bash
# Same-box A/B of a module constant: tools/ubench/knob_ab.sh <module> <NAME> "<v1> <v2> ..." <rounds> [bench args]
# e.g. tools/ubench/knob_ab.sh proteinbert_pytorch_replication_amd.ops.local_track WGRAD_CU_EIGHTHS "7 5" 2
mod=$1; name=$2; vals=$3; rounds=$4; shift 4
for r in $(seq "$rounds"); do
  for v in $vals; do
    out=$(timeout -k 10 300 python -u -c "
import sys, runpy, importlib
m = importlib.import_module('$mod')
setattr(m, '$name', $v)
sys.argv = ['bench.py'] + sys.argv[1:]
runpy.run_path('bench.py', run_name='__main__')
" "$@" 2>&1 | tail -1) || exit 1
    echo "$name=$v: $(echo "$out" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
