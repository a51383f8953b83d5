"""Summarise a rocprofv3 --kernel-trace --stats run: per-kernel totals (from *_kernel_stats.csv)
and, from *_kernel_trace.csv when present, the scan kernel's duration by merge-index bucket.
  python tools/prof_summary.py <rocprof output dir> > profiles/<name>.txt"""
import csv
import glob
import os
import sys

d = sys.argv[1]
stats = glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True)
for p in stats:
    rows = list(csv.DictReader(open(p)))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    print(f"# {os.path.relpath(p, d)}  total kernel time {tot / 1e6:.1f} ms")
    print(f"{'kernel':64s} {'calls':>8s} {'total ms':>10s} {'avg us':>10s} {'%':>6s}")
    for r in rows:
        print(f"{r['Name'][:64]:64s} {int(r['Calls']):8d} {float(r['TotalDurationNs']) / 1e6:10.1f} "
              f"{float(r['AverageNs']) / 1e3:10.2f} {float(r['Percentage']):6.2f}")
for p in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
    durs = []
    with open(p) as f:
        for r in csv.DictReader(f):
            if "zbpe_scan_pairs" in r.get("Kernel_Name", r.get("KernelName", "")):
                durs.append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    if not durs:
        continue
    print(f"\n# scan kernel launches: {len(durs)}; duration by launch-index bucket (us)")
    edges = [0, 10, 100, 1000, 5000, 10000, 20000, len(durs)]
    for lo, hi in zip(edges, edges[1:]):
        seg = durs[lo:hi]
        if seg:
            print(f"  launches {lo:6d}-{hi:6d}: avg {sum(seg) / len(seg) / 1e3:9.2f}  min {min(seg) / 1e3:9.2f}  max {max(seg) / 1e3:9.2f}")
