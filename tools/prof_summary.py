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

# timeline of the last merges: per-kernel durations and idle gaps between consecutive kernels
for p in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
    recs = []
    with open(p) as f:
        for r in csv.DictReader(f):
            name = r.get("Kernel_Name", r.get("KernelName", ""))
            recs.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name.split("(")[0].split("<")[0]))
    recs.sort()
    if len(recs) < 100:
        continue
    win = recs[-int(os.environ.get("TIMELINE_WINDOW", "30000")):]
    span = win[-1][1] - win[0][0]
    busy = sum(e - s for s, e, _ in win)
    per = {}
    gaps = {}
    for i, (s, e, n) in enumerate(win):
        per.setdefault(n, []).append(e - s)
        if i:
            gaps.setdefault(n, []).append(s - win[i - 1][1])
    nscan = len(per.get("void zbpe::zbpe_scan_pairs_t", per.get("zbpe::zbpe_scan_pairs_t", []))) or 1
    print(f"\n# timeline of the last {len(win)} kernels: span {span / 1e6:.1f} ms, busy {busy / 1e6:.1f} ms "
          f"({busy / span:.2f}), idle {(span - busy) / 1e6:.1f} ms")
    print(f"{'kernel':48s} {'calls':>7s} {'avg us':>8s} {'total ms':>9s} {'gap before avg us':>18s}")
    for n, v in sorted(per.items(), key=lambda kv: -sum(kv[1])):
        g = gaps.get(n, [0])
        print(f"{n[-48:]:48s} {len(v):7d} {sum(v) / len(v) / 1e3:8.2f} {sum(v) / 1e6:9.1f} {sum(g) / len(g) / 1e3:18.2f}")
