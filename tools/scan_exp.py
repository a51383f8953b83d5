"""Scan-kernel A/B: bench_scan over scan variants and pairs in one process (cdna_hip_programming.md rule 24).
  [VARIANTS=0,2,6] python tools/scan_exp.py [alternative libzbpe.so]"""
import os, sys, json
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "zig-bpe_amd"))
import zbpe
if len(sys.argv) > 1:
    zbpe.load_library(sys.argv[1])
text = zbpe.synth_corpus("words_utf8", 0x5EED0004, 1 << 30, threads=16)
e = zbpe.Engine(0)
e.upload(text)
pairs = {"rare": (1, 2), "e_sp": (101, 32), "sp_t": (32, 116), "t_h": (116, 104), "i_n": (105, 110)}
if os.environ.get("PAIRS"):  # name=a:b,...
    pairs = {kv.split("=")[0]: tuple(int(x) for x in kv.split("=")[1].split(":")) for kv in os.environ["PAIRS"].split(",")}
variants = [int(x) for x in os.environ.get("VARIANTS", "0,2,6,7").split(",")]
res = {}
for rnd in range(3):
    for v in variants:
        e.set_option("scan_variant", v)
        for name, (a, b) in pairs.items():
            ms, gbps = e.bench_scan(a, b, 5)
            k = f"v{v}"
            res.setdefault(k, {}).setdefault(name, 0)
            res[k][name] = max(res[k][name], round(gbps, 1))
for k, d in res.items():
    print(k, json.dumps(d))
