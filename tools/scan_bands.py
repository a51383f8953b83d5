"""Stream-form scan rate against pair density on the initial C4 stream (no holes, no block skipping):
pairs picked from the byte-pair histogram at target count/live densities, timed with zbpe_bench_scan
for each scan variant.
  python tools/scan_bands.py [--variants 0,1,2] [--n-bytes B]
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "zig-bpe_amd"))
import zbpe  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--n-bytes", type=int, default=1 << 30)
    p.add_argument("--variants", default="0")
    p.add_argument("--opt", action="append", default=[])
    a = p.parse_args()
    text = zbpe.synth_corpus("words_utf8", 0x5EED0004, a.n_bytes, threads=16)
    u = np.frombuffer(text, np.uint8)
    codes = u[:-1].astype(np.uint32) | (u[1:].astype(np.uint32) << 8)
    cnt = np.bincount(codes, minlength=65536)
    del codes
    n = len(u)
    e = zbpe.Engine(0)
    for kv in a.opt:
        k, v = kv.split("=")
        e.set_option(k, int(v))
    e.upload(text)
    picks = []
    self_pair = (np.arange(65536) & 0xFF) == (np.arange(65536) >> 8)
    for dens in (0.0, 0.0001, 0.0003, 0.0005, 0.001, 0.002, 0.005, 0.01, 0.03):
        dist = np.abs(cnt.astype(np.float64) - dens * n)
        dist[self_pair] = np.inf
        i = int(np.argmin(dist))
        picks.append((dens, i & 0xFF, i >> 8, int(cnt[i])))
    for v in (int(x) for x in a.variants.split(",")):
        e.set_option("scan_variant", v)
        for dens, x, y, c in picks:
            best = 0.0
            for _ in range(3):
                ms, gbps = e.bench_scan(x, y, 5)
                best = max(best, gbps)
            print(json.dumps({"variant": v, "density": dens, "pair": [x, y], "count": c, "GBps": round(best, 1)}), flush=True)
    e.close()


if __name__ == "__main__":
    main()
