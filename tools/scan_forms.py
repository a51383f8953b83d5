"""Per-form durations of the pair-scan kernel from a rocprofv3 kernel trace, matched launch by launch
to merges through bench.py's scan log (--scan-log-out: the probe train, the command's last train).

  rocprofv3 --kernel-trace --stats --output-format csv -d D -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu \
      --scan-log-out L.json
  python tools/scan_forms.py D L.json > profiles/<round>_c4_scan_forms.json

For the stream form it reports rocprof's average launch duration, the algorithmic bytes per launch
(2 B x live tokens) and their ratio against the 8 TB/s HBM peak -- the roofline that
bench.py's `roofline` measures with HIP events on the same launches. The list form is latency-bound
(reported: launches, average duration, walked entries when known). No-op launches (after a batch
halt) are counted separately.
"""
import csv
import glob
import json
import os
import sys

PEAK = 8000.0  # GB/s, MI355X_MICROARCH.md


def main():
    d, logp = sys.argv[1], sys.argv[2]
    files = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    if not files:
        sys.exit(f"no kernel trace under {d}")
    recs = []
    for p in files:
        with open(p) as f:
            for r in csv.DictReader(f):
                name = r.get("Kernel_Name", r.get("KernelName", ""))
                if "zbpe_scan_pairs_t" in name:
                    recs.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    recs.sort()
    L = json.load(open(logp))
    log, live = L["scan_log"], L["live"]
    if len(recs) < len(log):
        sys.exit(f"{len(recs)} scan dispatches in the trace, {len(log)} in the scan log")
    recs = recs[len(recs) - len(log):]
    g = {"stream": [], "list": [], "noop": []}
    for (s, e), x in zip(recs, log):
        if x < 0:
            g["noop"].append((e - s, 0))
        else:
            m, form = x >> 1, x & 1
            g["list" if form else "stream"].append((e - s, 2 * live[m]))
    out = {"kernel": "zbpe_scan_pairs_t", "source": os.path.relpath(files[0], d), "dispatches_matched": len(log)}
    for k, v in g.items():
        if not v:
            out[k] = {"launches": 0}
            continue
        ns = sum(a for a, _ in v)
        alg = sum(b for _, b in v)
        o = {"launches": len(v), "avg_us": ns / len(v) / 1e3, "total_ms": ns / 1e6}
        if k == "stream":
            o["alg_bytes_per_launch"] = alg / len(v)
            o["achieved_GBps"] = alg / ns if ns else 0.0
            o["frac_of_8TBps"] = o["achieved_GBps"] / PEAK
        out[k] = o
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
