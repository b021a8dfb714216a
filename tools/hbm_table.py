"""Per-kernel HBM traffic and achieved bandwidth of the headline step.

    python tools/hbm_table.py <fetch_dir> <write_dir> <kernel_stats.csv> [top]

<fetch_dir> / <write_dir>: rocprofv3 ``--pmc FETCH_SIZE`` and ``--pmc WRITE_SIZE`` passes
(``tools/gpu.sh pmc <tag> FETCH_SIZE`` ...; the two derived counters need 3 + 2 TCC counters, more than
one pass holds), both in KB per dispatch.  <kernel_stats.csv>: a ``--kernel-trace --stats`` run of the
same configuration for the time per call (the counter passes serialise kernels, so their durations are
not the step's).  Prints the top kernels by total time with MB read / written per call and the
achieved bandwidth (bytes past the L2: reads served by the 256 MB Infinity Cache count as fetched).
"""
import collections
import csv
import glob
import os
import sys


def per_kernel(d, counter):
    fs = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not fs:
        raise SystemExit(f"no counter_collection.csv under {d}")
    per_disp = collections.defaultdict(float)
    names = {}
    for f in fs:
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != counter:
                continue
            key = (f, r["Dispatch_Id"])
            per_disp[key] += float(r["Counter_Value"])
            names[key] = r["Kernel_Name"]
    agg = collections.defaultdict(list)
    for k, v in per_disp.items():
        agg[names[k]].append(v)
    return {n: sum(v) / len(v) / 1024.0 for n, v in agg.items()}     # KB -> MB per call


def main():
    fdir, wdir, stats = sys.argv[1:4]
    top = int(sys.argv[4]) if len(sys.argv) > 4 else 12
    fetch = per_kernel(fdir, "FETCH_SIZE")
    write = per_kernel(wdir, "WRITE_SIZE")
    rows = []
    for r in csv.DictReader(open(stats)):
        rows.append((float(r["TotalDurationNs"]), int(r["Calls"]), float(r["AverageNs"]) / 1e3, r["Name"]))
    rows.sort(reverse=True)
    print(f"{'kernel':60s} {'calls':>6s} {'read MB':>8s} {'write MB':>8s} {'us/call':>8s} {'TB/s':>6s}")
    for tot, calls, us, name in rows[:top]:
        f = fetch.get(name)
        w = write.get(name)
        if f is None or w is None:
            print(f"{name[:60]:60s} {calls:6d} {'-':>8s} {'-':>8s} {us:8.1f} {'-':>6s}")
            continue
        print(f"{name[:60]:60s} {calls:6d} {f:8.1f} {w:8.1f} {us:8.1f} {(f + w) / us:6.2f}")


if __name__ == "__main__":
    main()
