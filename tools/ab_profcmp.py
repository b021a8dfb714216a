"""Compare two rocprofv3 kernel_stats.csv files (per-call average by kernel): python tools/ab_profcmp.py A B"""
import csv
import glob
import os
import sys


def load(d):
    f = max(glob.glob(f"{d}/**/*kernel_stats.csv", recursive=True), key=os.path.getmtime)
    return {r["Name"][:70]: (float(r["AverageNs"]) / 1e3, int(r["Calls"]), float(r["TotalDurationNs"]) / 1e3)
            for r in csv.DictReader(open(f))}


a, b = load(sys.argv[1]), load(sys.argv[2])
rows = sorted(set(a) | set(b), key=lambda k: -max(a.get(k, (0, 0, 0))[2], b.get(k, (0, 0, 0))[2]))
print(f"{'kernel':70s} {'A us':>8s} {'B us':>8s} {'diff':>7s}")
for k in rows[:25]:
    x, y = a.get(k, (0, 0, 0))[0], b.get(k, (0, 0, 0))[0]
    print(f"{k:70s} {x:8.1f} {y:8.1f} {(x - y):7.1f}")
