"""FETCH_SIZE calibration for the scan kernel's access pattern (MI355X_MICROARCH.md: "calibrate on a
known byte count in your own access pattern"): zbpe_bench_scan streams the whole uploaded stream
(no block skipping), so a pair that never occurs reads exactly 2 B per slot and nothing else.
  rocprofv3 --pmc FETCH_SIZE --kernel-include-regex zbpe_scan_pairs --output-format csv -d D -o run -- \
      python3 tools/pmc_calib.py
Launch order: for each variant in VARIANTS, 3 launches of each pair in PAIRS (tools/pmc_calib.sh)."""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "zig-bpe_amd"))
import zbpe  # noqa: E402

VARIANTS = (0, 6, 2)  # non-temporal loads, plain loads, compacted phase 2 (engine.hip kScanVariants)
PAIRS = ((1, 2), (101, 32))  # never occurs; (e, ' '), the densest C4 pair
n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 30
e = zbpe.Engine(0)
e.upload(zbpe.synth_corpus("words_utf8", 0x5EED0004, n, threads=16))
out = []
for v in VARIANTS:
    e.set_option("scan_variant", v)
    for a, b in PAIRS:
        ms, gbps = e.bench_scan(a, b, 3)
        out.append({"variant": v, "pair": [a, b], "stream_bytes": 2 * n, "avg_ms": ms, "GBps": gbps})
print(json.dumps(out))
