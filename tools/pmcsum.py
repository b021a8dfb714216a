"""Summarise rocprofv3 --pmc passes (gpurun_out/<dir>/runc/*_counter_collection.csv) per kernel."""
import collections
import csv
import glob
import sys

res = collections.defaultdict(lambda: collections.defaultdict(list))
for d in sys.argv[1:]:
    fs = glob.glob(f"gpurun_out/{d}/**/*counter_collection.csv", recursive=True)
    if not fs:
        print("missing", d)
        continue
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    names = {}
    for r in csv.DictReader(open(fs[0])):
        agg[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
        names[r["Dispatch_Id"]] = r["Kernel_Name"]
    for k, v in agg.items():
        for c, x in v.items():
            res[names[k][:48]][c].append(x)
for n, v in sorted(res.items()):
    m = {c: sum(x) / len(x) for c, x in v.items()}
    clk = m.get("GRBM_GUI_ACTIVE", 0) / 8
    if clk < 20000:
        continue
    mf = m.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / 1024 / clk
    nm = max(1.0, m.get("SQ_INSTS_MFMA", 1))
    wc = max(1.0, m.get("SQ_WAVE_CYCLES", 1))
    print(f"{n:48s} cyc {clk:9.0f} mfma_busy {mf:5.2f} valu/mfma {m.get('SQ_INSTS_VALU', 0) / nm:6.2f} "
          f"lds/mfma {m.get('SQ_INSTS_LDS', 0) / nm:5.2f} wait_any {m.get('SQ_WAIT_ANY', 0) / wc:4.2f} "
          f"wait_inst {m.get('SQ_WAIT_INST_ANY', 0) / wc:4.2f} active_valu/clk/simd "
          f"{m.get('SQ_ACTIVE_INST_VALU', 0) * 4 / max(1.0, clk) / 1024:5.2f}")
