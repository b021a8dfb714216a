R=$GRAFT_REPO_ROOT
cd $R
for b in 512 1024 2048; do
  timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 --batch $b > gpurun_out/bs_$b.json 2> gpurun_out/bs_$b.err || { tail -5 gpurun_out/bs_$b.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/bs_$b.json'));print($b, d['value'], d['ms_per_step'])"
done
