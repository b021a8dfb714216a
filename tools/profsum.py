"""Summarise a rocprofv3 kernel_stats.csv: top kernels by total time (per-step if --steps given)."""
import csv, sys
path = sys.argv[1]
steps = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
rows = list(csv.DictReader(open(path)))
tot = sum(float(r['TotalDurationNs']) for r in rows)
print(f"total {tot/1e6:.2f} ms over profile ({tot/1e6/steps:.3f} ms/step for {steps:g} steps)")
for r in rows[:int(sys.argv[3]) if len(sys.argv) > 3 else 30]:
    print(f"{float(r['TotalDurationNs'])/1e6/steps:8.3f} ms/step {int(r['Calls'])/steps:7.1f} calls/step "
          f"{float(r['AverageNs'])/1e3:9.1f} us/call {float(r['Percentage']):6.2f}%  {r['Name'][:90]}")
