"""GPU idle analysis of a rocprofv3 kernel_trace.csv: per step (delimited by the Adam kernel) the span,
the UNION of kernel intervals (concurrent streams counted once) and the largest idle gaps with the
kernels on either side.   python tools/gpu_idle.py trace.csv [top_gaps]"""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r['Start_Timestamp']))
top = int(sys.argv[2]) if len(sys.argv) > 2 else 8
iv = [(int(r['Start_Timestamp']), int(r['End_Timestamp']), r['Kernel_Name'][:50]) for r in rows]
idx = [i for i, r in enumerate(rows) if 'adam_flat' in r['Kernel_Name']]
for a, b in zip(idx[:-1], idx[1:]):
    seg = iv[a + 1:b + 1]
    t0, t1 = seg[0][0], max(e for _, e, _ in seg)
    busy, cur_s, cur_e, gaps, prev = 0, seg[0][0], seg[0][1], [], seg[0][2]
    for s, e, n in seg[1:]:
        if s > cur_e:
            busy += cur_e - cur_s
            gaps.append((s - cur_e, prev, n))
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
        prev = n if e >= cur_e else prev
    busy += cur_e - cur_s
    print(f"step span {(t1 - t0) / 1e6:.3f} ms  busy(union) {busy / 1e6:.3f} ms  idle {(t1 - t0 - busy) / 1e3:.0f} us"
          f"  gaps {len(gaps)}")
last = gaps
print("largest gaps of the last step:")
for g, p, n in sorted(last, reverse=True)[:top]:
    print(f"  {g / 1e3:7.1f} us  after {p}  before {n}")
