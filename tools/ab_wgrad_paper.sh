R=$GRAFT_REPO_ROOT; cd $R
for i in 1 2; do for r in 64 56; do
  PBX_WGRAD_R=$r timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --semantics paper > gpurun_out/p_$r.json 2>/dev/null || exit 1
  echo "paper R=$r $(python3 -c "import json;d=json.load(open('gpurun_out/p_$r.json'));print(d['value'])")"
done; done
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/def.json 2>/dev/null && echo "default $(python3 -c "import json;d=json.load(open('gpurun_out/def.json'));print(d['value'])")"
