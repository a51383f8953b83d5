"""Scan-kernel rate vs key-token density (no profiler): zbpe_bench_scan over the whole C4 stream for
pairs whose first token is absent, frequent or the most frequent, and which occur rarely or densely.
  python tools/scan_density.py [n_bytes]"""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "zig-bpe_amd"))
import zbpe  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 30
variants = [int(v) for v in sys.argv[2].split(",")] if len(sys.argv) > 2 else [0]
e = zbpe.Engine(0)
e.upload(zbpe.synth_corpus("words_utf8", 0x5EED0004, n, threads=16))
pairs = {"absent_key(1,2)": (1, 2), "e_key_absent_pair(101,1)": (101, 1), "space_key_absent(32,1)": (32, 1),
         "e_x(101,120)": (101, 120), "dense(101,32)": (101, 32)}
for v in variants:
    e.set_option("scan_variant", v)
    for name, (a, b) in pairs.items():
        best = 0
        for _ in range(3):
            ms, gbps = e.bench_scan(a, b, 5)
            best = max(best, gbps)
        print(json.dumps({"variant": v, "pair": name, "GBps": round(best, 1)}), flush=True)
