"""HBM traffic of the pair-scan kernel from rocprofv3 PMC passes, matched launch by launch to merges.

  rocprofv3 --pmc FETCH_SIZE --kernel-include-regex zbpe_scan_pairs --output-format csv -d D1 -o run -- \
      python3 bench.py --steps 1 --warmup 0 --no-cpu --scan-log-out L1.json
  rocprofv3 --pmc WRITE_SIZE ... -d D2 ... --scan-log-out L2.json
  python tools/pmc_traffic.py --fetch D1 --fetch-log L1.json --write D2 --write-log L2.json > profiles/<round>_pmc_traffic.json

Corrections (MI355X_MICROARCH.md "HBM [CDNA4]"): FETCH_SIZE and WRITE_SIZE are in KiB; on gfx950
FETCH_SIZE reports 1/2 of the bytes of a wide coalesced (16 B/lane) streaming read, so it is doubled.
Infinity-Cache hits are counted, not excluded (the C4 stream is 2 GiB, far past the 256 MiB L3).

The scan log (Engine.scan_log) has one entry per scan launch in launch order (2 * merge + form,
-1 = a no-op launch after a batch halt), so the k-th profiled dispatch of the kernel is log entry k.
Reported per launch, like bench.py's roofline: over all stream-form launches, over the timed ones
(every 8th merge, the launches bench.py's `achieved` is measured on), and over list-form launches.
"""
import argparse
import csv
import glob
import json
import os
import sys

KERNEL = "zbpe_scan_pairs"


def per_dispatch(d, counter):
    """[(dispatch id, value)] of `counter` for the scan kernel, in dispatch order."""
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        sys.exit(f"no *counter_collection.csv under {d}")
    vals = {}
    for p in files:
        with open(p) as f:
            for r in csv.DictReader(f):
                name = r.get("Kernel_Name", r.get("KernelName", ""))
                if KERNEL not in name or r.get("Counter_Name") != counter:
                    continue
                did = int(r.get("Dispatch_Id", r.get("Correlation_Id")))
                vals[did] = vals.get(did, 0.0) + float(r["Counter_Value"])
    return [vals[k] for k in sorted(vals)]


def summarise(values, log, live, scale):
    # bench.py trains several times (warm-up, timed steps, the probe train); the scan log is the probe
    # train's, the last train of the command: its launches are the last len(log) dispatches
    if len(values) < len(log):
        sys.exit(f"{len(values)} profiled scan dispatches but {len(log)} scan-log entries: cannot match")
    values = values[len(values) - len(log):]
    groups = {"stream": [], "stream_timed": [], "list": [], "noop": []}
    for v, e in zip(values, log):
        if e < 0:
            groups["noop"].append((v, 0))
            continue
        merge, form = e >> 1, e & 1
        alg = 2 * live[merge]
        if form:
            groups["list"].append((v, alg))
        else:
            groups["stream"].append((v, alg))
            if (merge + 256) % 8 == 0:
                groups["stream_timed"].append((v, alg))
    out = {}
    for k, g in groups.items():
        if not g:
            out[k] = {"launches": 0}
            continue
        b = sum(v for v, _ in g) * scale / len(g)
        a = sum(x for _, x in g) / len(g)
        out[k] = {"launches": len(g), "bytes_per_launch": b, "alg_bytes_per_launch": a,
                  "bytes_over_alg": b / a if a else None}
    return out


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--fetch", required=True)
    p.add_argument("--fetch-log", required=True)
    p.add_argument("--write", default="")
    p.add_argument("--write-log", default="")
    a = p.parse_args()
    res = {"kernel": "zbpe_scan_pairs_t", "source": "rocprofv3 --pmc, one pass per counter, bench.py --steps 1 --warmup 0 --no-cpu (the probe train: the last train of the command)",
           "correction": "FETCH_SIZE KiB x 1024 x 2 (gfx950 wide-read undercount); WRITE_SIZE KiB x 1024"}
    fl = json.load(open(a.fetch_log))
    res["read"] = summarise(per_dispatch(a.fetch, "FETCH_SIZE"), fl["scan_log"], fl["live"], 2 * 1024)
    if a.write:
        wl = json.load(open(a.write_log))
        if wl["scan_log"] != fl["scan_log"]:
            sys.exit("the two passes launched different scan sequences")
        res["write"] = summarise(per_dispatch(a.write, "WRITE_SIZE"), wl["scan_log"], wl["live"], 1024)
    t = {}
    for k in ("stream", "stream_timed", "list"):
        r = res["read"][k]
        if not r["launches"]:
            continue
        w = res.get("write", {}).get(k, {}).get("bytes_per_launch", 0.0)
        t[k] = {"launches": r["launches"], "hbm_bytes_per_launch": r["bytes_per_launch"] + w,
                "alg_bytes_per_launch": r["alg_bytes_per_launch"],
                "hbm_over_alg": (r["bytes_per_launch"] + w) / r["alg_bytes_per_launch"]}
    res["traffic"] = t
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
