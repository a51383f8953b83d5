"""C5 (BASELINE.json configs[4]): encode 100 M chars with the C4 merges (vocab 32000) on one GPU.

  python tools/encode_bench.py [--n-bytes 100000000] [--train-bytes 2^30] [--vocab 32000] [--check-bytes 200000]

Trains C4 (seed 0x5EED0004) for the merges, then times zbpe_encode of a C5 text (same generator,
seed 0x5EED0005, host buffer in and out, PCIe included) and checks a prefix against the oracle's
linear encode. Prints one JSON line.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "zig-bpe_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import zbpe  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--n-bytes", type=int, default=100_000_000)
    p.add_argument("--train-bytes", type=int, default=1 << 30)
    p.add_argument("--vocab", type=int, default=32000)
    p.add_argument("--check-bytes", type=int, default=200_000)
    p.add_argument("--reps", type=int, default=2)
    p.add_argument("--opt", action="append", default=[], help="engine option k=v applied before encode (repeatable)")
    a = p.parse_args()
    e = zbpe.Engine(0)
    e.upload(zbpe.synth_corpus("words_utf8", 0x5EED0004, a.train_bytes, threads=16))
    merges, counts, st = e.train_resident(a.vocab)
    text = zbpe.synth_corpus("words_utf8", 0x5EED0005, a.n_bytes, threads=16)
    for kv in a.opt:
        k, v = kv.split("=")
        e.set_option(k, int(v))
    times = []
    out = None
    for _ in range(a.reps):
        t = time.perf_counter()
        out = e.encode(merges, text)
        times.append(time.perf_counter() - t)
    best = min(times)
    res = {"metric": "encode chars/s (C5: 100 M chars, C4 merges)", "value": a.n_bytes / best, "unit": "chars/s",
           "seconds": best, "merges": int(len(merges)), "tokens_out": int(len(out)), "reps": a.reps,
           "opts": a.opt}
    if a.check_bytes:
        import oracle as O
        ref = O.encode(merges, text[: a.check_bytes])
        dev = e.encode(merges, text[: a.check_bytes])
        res["prefix_check"] = {"bytes": a.check_bytes, "equal": bool(np.array_equal(np.asarray(ref), dev))}
    print(json.dumps(res))
    e.close()


if __name__ == "__main__":
    main()
