# Same-box A/B of the bench step: the in-tree library vs tools/ubench/abl/libpbx_<name>.so, alternated.
# usage: bash tools/ab_bench.sh <name> [rounds] [extra bench args]
R=$GRAFT_REPO_ROOT
cd $R
name=$1; rounds=${2:-2}; shift 2
for i in $(seq 1 $rounds); do
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 "$@" > gpurun_out/ab_new_$i.json 2> gpurun_out/ab_new_$i.err || exit 1
  PBX_HIP_LIB=tools/ubench/abl/libpbx_$name.so timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 "$@" > gpurun_out/ab_${name}_$i.json 2> gpurun_out/ab_${name}_$i.err || exit 1
done
grep -h '"value"' gpurun_out/ab_*.json | python3 -c "
import json,sys
for l in sys.stdin: d=json.loads(l); print(d['value'], d['ms_per_step'])"
