"""Per-kernel averages of rocprofv3 PMC counters over the LAST N dispatches of each kernel (the late merges of a C4
train): python tools/pmc_kernel_summary.py <rocprofv3 -d dir> [N]"""
import collections
import csv
import glob
import json
import sys

d = sys.argv[1]
N = int(sys.argv[2]) if len(sys.argv) > 2 else 10000
f = glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)
if not f:
    sys.exit(f"no counter csv under {d}")
rows = list(csv.DictReader(open(f[0])))
by = collections.defaultdict(lambda: collections.defaultdict(dict))  # kernel -> dispatch -> counter -> value
for r in rows:
    k = r.get("Kernel_Name", r.get("KernelName", ""))[:40]
    dd = by[k][int(r.get("Dispatch_Id", r.get("Correlation_Id")))]
    dd[r["Counter_Name"]] = dd.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])  # (rows per instance summed)
out = {}
for k, disp in by.items():
    ids = sorted(disp)[-N:]
    names = sorted({c for i in ids for c in disp[i]})
    out[k] = {"dispatches": len(ids), **{c: sum(disp[i].get(c, 0.0) for i in ids) / len(ids) for c in names}}
print(json.dumps(out, indent=1))
