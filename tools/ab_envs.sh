# Same-box comparison of the bench step under several environment settings, round-robin.
# usage: bash tools/ab_envs.sh <rounds> "<env A>" "<env B>" ...
R=$GRAFT_REPO_ROOT
cd $R
rounds=$1; shift
for i in $(seq 1 $rounds); do
  k=0
  for envs in "$@"; do
    k=$((k+1))
    env $envs timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 > gpurun_out/abs_${k}_$i.json 2> gpurun_out/abs_${k}_$i.err || exit 1
    echo "[$envs] $(python3 -c "import json;d=json.load(open('gpurun_out/abs_${k}_$i.json'));print(d['value'], d['ms_per_step'])")"
  done
done
