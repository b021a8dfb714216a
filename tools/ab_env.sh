# Same-box A/B of the bench step under two environment settings, alternated.
# usage: bash tools/ab_env.sh "<env A>" "<env B>" [rounds]
R=$GRAFT_REPO_ROOT
cd $R
A=$1; B=$2; rounds=${3:-2}
for i in $(seq 1 $rounds); do
  for tag in A B; do
    envs=$([ $tag = A ] && echo "$A" || echo "$B")
    env $envs timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/abe_${tag}_$i.json 2> gpurun_out/abe_${tag}_$i.err || exit 1
    echo "$tag [$envs] $(python3 -c "import json;d=json.load(open('gpurun_out/abe_${tag}_$i.json'));print(d['value'], d['ms_per_step'])")"
  done
done
