"""Raw per-kernel counter means from rocprofv3 --pmc csv output:
    python tools/ubench/pmc_raw.py [--match SUBSTRING] <dir>..."""
import collections
import csv
import glob
import sys

args = sys.argv[1:]
match = ""
if args[:1] == ["--match"]:
    match, args = args[1], args[2:]
for d in args:
    fs = glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)
    if not fs:
        print("missing", d)
        continue
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    names = {}
    for r in csv.DictReader(open(fs[0])):
        agg[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
        names[r["Dispatch_Id"]] = r["Kernel_Name"]
    per = collections.defaultdict(lambda: collections.defaultdict(list))
    for k, v in agg.items():
        for c, x in v.items():
            per[names[k][:40]][c].append(x)
    for n, v in sorted(per.items()):
        if match not in n:
            continue
        print(d, n, " ".join(f"{c}={sum(x) / len(x):.4g}" for c, x in sorted(v.items())))
