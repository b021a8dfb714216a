"""Per-kernel SQ counter summary of a rocprofv3 --pmc pass (any program):
    python tools/ubench/pmc_kernels.py <dir-with-counter_collection.csv> [min_cycles]
mfma_busy = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMD-cycles), the rest per wave-cycle / per MFMA."""
import collections
import csv
import glob
import os
import sys

d = sys.argv[1]
mn = float(sys.argv[2]) if len(sys.argv) > 2 else 5000
f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)[0]
agg = collections.defaultdict(lambda: collections.defaultdict(float))
names = {}
for r in csv.DictReader(open(f)):
    agg[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
    names[r["Dispatch_Id"]] = r["Kernel_Name"]
res = collections.defaultdict(list)
for k, v in agg.items():
    res[names[k][:44]].append(v)
for n, vs in sorted(res.items()):
    m = {c: sum(v.get(c, 0.0) for v in vs) / len(vs) for c in vs[0]}
    clk = m.get("GRBM_GUI_ACTIVE", 0) / 8
    if clk < mn:
        continue
    wc = max(1.0, m.get("SQ_WAVE_CYCLES", 1))
    nm = max(1.0, m.get("SQ_INSTS_MFMA", 1))
    print(f"{n:44s} clk {clk:8.0f} mfma_busy {m.get('SQ_VALU_MFMA_BUSY_CYCLES', 0) / 1024 / clk:5.2f} "
          f"valu/mfma {m.get('SQ_INSTS_VALU', 0) / nm:6.2f} lds/mfma {m.get('SQ_INSTS_LDS', 0) / nm:5.2f} "
          f"wait_any {m.get('SQ_WAIT_ANY', 0) / wc:4.2f} wait_inst {m.get('SQ_WAIT_INST_ANY', 0) / wc:4.2f} "
          f"valu_active {m.get('SQ_ACTIVE_INST_VALU', 0) / wc:4.2f}")
