"""Per-queue timeline of one step from a rocprofv3 kernel_trace.csv: busy time per queue, the main
queue's idle gaps (what it waited on), and the kernels that ran concurrently with nothing on the main
queue.   python tools/critpath.py trace.csv [step_index_from_end]"""
import collections
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r['Start_Timestamp']))
k = int(sys.argv[2]) if len(sys.argv) > 2 else 2
idx = [i for i, r in enumerate(rows) if 'adam_flat' in r['Kernel_Name']]
a, b = idx[-1 - k], idx[-k]
seg = rows[a + 1:b + 1]
t0 = int(seg[0]['Start_Timestamp'])
t1 = int(seg[-1]['End_Timestamp'])
q = collections.defaultdict(list)
for r in seg:
    q[r['Queue_Id']].append(r)
print(f"step span {(t1 - t0) / 1e3:.1f} us, {len(seg)} kernels")
main = max(q, key=lambda x: len(q[x]))
for qid, rs in q.items():
    busy = sum(int(r['End_Timestamp']) - int(r['Start_Timestamp']) for r in rs)
    print(f"queue {qid}{' (main)' if qid == main else ''}: {len(rs)} kernels, busy {busy / 1e3:.1f} us")
rs = q[main]
gaps = []
for p, n in zip(rs[:-1], rs[1:]):
    g = int(n['Start_Timestamp']) - int(p['End_Timestamp'])
    gaps.append((g, p['Kernel_Name'][:50], n['Kernel_Name'][:50]))
print(f"main-queue idle total {sum(g for g, _, _ in gaps) / 1e3:.1f} us; largest gaps:")
for g, p, n in sorted(gaps, reverse=True)[:15]:
    print(f"  {g / 1e3:7.1f} us  after {p}  ->  {n}")
print("main-queue kernels in order (us, concurrent aux-queue kernels overlapping):")
aux = [r for r in seg if r['Queue_Id'] != main]
for r in rs:
    s, e = int(r['Start_Timestamp']), int(r['End_Timestamp'])
    ov = [x['Kernel_Name'][:28] for x in aux if int(x['Start_Timestamp']) < e and int(x['End_Timestamp']) > s]
    print(f"  {(s - t0) / 1e3:8.1f} {(e - s) / 1e3:7.1f}  {r['Kernel_Name'][:45]:45s} | {', '.join(sorted(set(ov)))[:90]}")
print("aux-queue kernels in order (queue, start us, duration us):")
for r in sorted(aux, key=lambda x: int(x['Start_Timestamp'])):
    s, e = int(r['Start_Timestamp']), int(r['End_Timestamp'])
    print(f"  q{r['Queue_Id']:>3s} {(s - t0) / 1e3:8.1f} {(e - s) / 1e3:7.1f}  {r['Kernel_Name'][:60]}")
