"""Per-step GPU span / busy time from a rocprofv3 kernel_trace.csv (steps delimited by the Adam kernel),
plus per-kernel mean duration over the last N steps.   python tools/stepspan.py trace.csv [N]"""
import collections
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r['Start_Timestamp']))
last = int(sys.argv[2]) if len(sys.argv) > 2 else 5
idx = [i for i, r in enumerate(rows) if 'adam_flat' in r['Kernel_Name']]
per = collections.defaultdict(list)
for a, b in list(zip(idx[:-1], idx[1:])):
    seg = rows[a + 1:b + 1]
    t0, t1 = int(seg[0]['Start_Timestamp']), int(seg[-1]['End_Timestamp'])
    busy = sum(int(r['End_Timestamp']) - int(r['Start_Timestamp']) for r in seg)
    print(f"step span {(t1 - t0) / 1e6:.3f} ms  busy {busy / 1e6:.3f} ms  kernels {len(seg)}")
for a, b in list(zip(idx[:-1], idx[1:]))[-last:]:
    for r in rows[a + 1:b + 1]:
        per[r['Kernel_Name'][:60]].append(int(r['End_Timestamp']) - int(r['Start_Timestamp']))
tot = sum(sum(v) for v in per.values()) / last
print(f"mean over last {last} steps: {tot / 1e6:.3f} ms")
for k, v in sorted(per.items(), key=lambda kv: -sum(kv[1]))[:25]:
    print(f"{sum(v) / last / 1e3:9.1f} us/step {len(v) / last:5.1f} calls {sum(v) / len(v) / 1e3:8.1f} us/call  {k}")
