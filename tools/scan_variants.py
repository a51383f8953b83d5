"""A/B the scan-kernel variants (engine.hip kScanVariants) on one process and device
(cdna_hip_programming.md rule 24: interleaved rounds in ONE process).
  python tools/scan_variants.py [n_bytes]"""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "zig-bpe_amd"))
import zbpe  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 30
text = zbpe.synth_corpus("words_utf8", 0x5EED0004, n, threads=16)
e = zbpe.Engine(0)
e.upload(text)
pairs = {"rare(1,2)": (1, 2), "e_space(101,32)": (101, 32), "common(32,116)": (32, 116)}
res = {}
for rnd in range(3):
    for v in range(5):
        e.set_option("scan_variant", v)
        for name, (a, b) in pairs.items():
            ms, gbps = e.bench_scan(a, b, 6)
            res.setdefault(f"v{v} {name}", []).append(round(gbps, 1))
for k, x in res.items():
    print(k.ljust(28), "GB/s per round:", x, "best", max(x))
print(json.dumps({k: max(x) for k, x in res.items()}))
