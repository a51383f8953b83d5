"""Full pair-histogram kernel (zbpe_pair_hist) timing on C4 states: t = 0 and after K merges.

  python tools/hist_bench.py [--n-bytes B] [--at 0 --at 20000 ...] [--reps R]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "zig-bpe_amd"))
import zbpe  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--n-bytes", type=int, default=1 << 30)
    p.add_argument("--at", type=int, action="append", default=[])
    p.add_argument("--reps", type=int, default=5)
    p.add_argument("--opt", action="append", default=[], help="engine option k=v (e.g. dense_hist=0)")
    a = p.parse_args()
    e = zbpe.Engine(0)
    for kv in a.opt:
        k, v = kv.split("=")
        e.set_option(k, int(v))
    e.upload(zbpe.synth_corpus("words_utf8", 0x5EED0004, a.n_bytes, threads=16))
    for k in a.at or [0, 20000]:
        _, _, st = e.train_resident(256 + k)
        r = e.bench_recount(a.reps)
        r.update(merges=k, distinct_pairs=int(st.distinct_pairs), frac=r["GBps"] / 8000.0, opts=a.opt)
        print(json.dumps(r), flush=True)
    e.close()


if __name__ == "__main__":
    main()
