"""A/B the stream-scan kernel variants (engine.hip kScanVariants) over pairs of different key density,
in one process and device (cdna_hip_programming.md rule 24: interleaved rounds in ONE process).

  [VARIANTS=0,2,6] [PAIRS=name=a:b,...] python tools/scan_variants.py [n_bytes] [alternative libzbpe.so]

Prints the best GB/s (2 B per stream slot / launch time, zbpe_bench_scan) per variant and pair over 3 rounds.
"""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "zig-bpe_amd"))
import zbpe  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 30
if len(sys.argv) > 2:
    zbpe.load_library(sys.argv[2])
text = zbpe.synth_corpus("words_utf8", 0x5EED0004, n, threads=16)
e = zbpe.Engine(0)
e.upload(text)
pairs = {"rare(1,2)": (1, 2), "e_space(101,32)": (101, 32), "common(32,116)": (32, 116), "t_h(116,104)": (116, 104),
         "i_n(105,110)": (105, 110)}
if os.environ.get("PAIRS"):  # name=a:b,...
    pairs = {kv.split("=")[0]: tuple(int(x) for x in kv.split("=")[1].split(":")) for kv in os.environ["PAIRS"].split(",")}
variants = [int(x) for x in os.environ.get("VARIANTS", "0,1,2,3,4,5,6").split(",")]
res = {}
for rnd in range(3):
    for v in variants:
        e.set_option("scan_variant", v)
        for name, (a, b) in pairs.items():
            ms, gbps = e.bench_scan(a, b, 6)
            res.setdefault(f"v{v} {name}", []).append(round(gbps, 1))
for k, x in res.items():
    print(k.ljust(28), "GB/s per round:", x, "best", max(x))
print(json.dumps({k: max(x) for k, x in res.items()}))
