# per-GPU batch sweep of the headline step on the current build (B=512 is the preset)
cd $GRAFT_REPO_ROOT
for r in 1 2; do for b in 512 576 608 768; do
  timeout -k 10 200 python -u bench.py --batch $b --steps 30 > gpurun_out/bs_${b}_$r.json 2>/dev/null || exit 1
  echo "B=$b run $r: $(python3 -c "import json;d=json.load(open('gpurun_out/bs_${b}_$r.json'));print(d['value'], d['ms_per_step'])")"
done; done
