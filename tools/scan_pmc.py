"""One pair's stream-form scan launches on the fresh C4 stream, for a rocprofv3 --pmc pass:
  rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY ... --kernel-include-regex zbpe_scan_pairs -d D -o run -- \
      python3 tools/scan_pmc.py --pair 112,97 --reps 20
  python3 tools/scan_pmc.py --summarise D   (per-counter sums over the launches, per launch)"""
import argparse
import csv
import glob
import json
import os
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--pair", default="")
    p.add_argument("--reps", type=int, default=20)
    p.add_argument("--n-bytes", type=int, default=1 << 30)
    p.add_argument("--summarise", default="")
    p.add_argument("--variant", type=int, default=-1, help="option scan_variant (7: the batched form)")
    a = p.parse_args()
    if a.summarise:
        tot, launches = defaultdict(float), set()
        for f in glob.glob(os.path.join(a.summarise, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                launches.add(r.get("Dispatch_Id") or r.get("Correlation_Id"))
                tot[r["Counter_Name"]] += float(r["Counter_Value"])
        n = max(len(launches), 1)
        print(json.dumps({"launches": n, "per_launch": {k: v / n for k, v in sorted(tot.items())}}))
        return
    sys.path.insert(0, os.path.join(ROOT, "zig-bpe_amd"))
    import zbpe
    x, y = (int(v) for v in a.pair.split(","))
    e = zbpe.Engine(0)
    e.upload(zbpe.synth_corpus("words_utf8", 0x5EED0004, a.n_bytes, threads=16))
    if a.variant >= 0:
        e.set_option("scan_variant", a.variant)
    ms, gbps = e.bench_scan(x, y, a.reps)
    print(json.dumps({"pair": [x, y], "ms": ms, "GBps": gbps}))
    e.close()


if __name__ == "__main__":
    main()
