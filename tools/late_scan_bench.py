"""Late-phase pair-scan microbenchmark (zbpe_bench_train_scan): train C4 to each vocab size, then time
the next merge's scan launched as training would, on several grids. One JSON line per (vocab, grid).

  python tools/late_scan_bench.py [--vocab 8000 20000 31000] [--grid 0 16 64] [--reps 50]
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
    p.add_argument("--seed", type=int, default=0x5EED0004)
    p.add_argument("--vocab", type=int, nargs="+", default=[8000, 20000, 31000])
    p.add_argument("--grid", type=int, nargs="+", default=[0, 16, 64])
    p.add_argument("--reps", type=int, default=50)
    p.add_argument("--opt", action="append", default=[])
    a = p.parse_args()
    e = zbpe.Engine(0)
    for o in a.opt:
        k, v = o.split("=")
        e.set_option(k, int(v))
    e.upload(zbpe.synth_corpus("words_utf8", a.seed, a.n_bytes, threads=16))
    for v in a.vocab:
        m, c, st = e.train_resident(v)
        for g in a.grid:
            r = e.bench_train_scan(a.reps, g)
            r.update({"vocab": v, "grid": g, "next_count": int(c[-1]) if len(c) else 0, "lib": os.environ.get("ZBPE_LIB", "")})
            print(json.dumps(r), flush=True)
    e.close()


if __name__ == "__main__":
    main()
