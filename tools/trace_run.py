"""Per-merge timing trace of one C4 train (option "trace"), summarised by merge-index buckets.

  python tools/trace_run.py [--n-bytes B] [--vocab V] [--opt name=value ...] [--out gpurun_out/trace.npy]

Columns: zbpe.TRACE_COLUMNS. Prints, per bucket of merges: mean count, live tokens, fraction of the
stream the scan streamed, mean scan / replace / select / wall ms, and the bucket's share of the wall.
"""
import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "zig-bpe_amd"))
import zbpe  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--n-bytes", type=int, default=1 << 30)
    p.add_argument("--vocab", type=int, default=32000)
    p.add_argument("--seed", type=int, default=0x5EED0004)
    p.add_argument("--opt", action="append", default=[])
    p.add_argument("--out", default="")
    p.add_argument("--buckets", type=int, default=16)
    a = p.parse_args()
    eng = zbpe.Engine(0)
    for o in a.opt:
        k, v = o.split("=")
        eng.set_option(k, int(v))
    eng.set_option("trace", 1)
    text = zbpe.synth_corpus("words_utf8", a.seed, a.n_bytes, threads=16)
    eng.upload(text)
    eng.train_resident(a.vocab)  # warm
    t = time.perf_counter()
    m, c, st = eng.train_resident(a.vocab)
    wall = time.perf_counter() - t
    tr = eng.trace()
    if a.out:
        np.save(a.out, tr)
    print(f"opts {a.opt}: {len(m)} merges in {wall:.3f} s = {len(m) / wall:.1f} merges/s; "
          f"scan {st.scan_kernel_s:.3f} s, replace {st.replace_pair_s:.3f} s, select {st.sort_pairs_s:.3f} s")
    C = {k: i for i, k in enumerate(zbpe.TRACE_COLUMNS)}
    tot_wall = tr[:, C["wall_ms"]].sum()
    print("%-13s %9s %11s %6s %8s %8s %8s %8s %6s %5s" % ("merges", "count", "live", "strm", "scan", "repl", "sel",
                                                         "wall", "share", "ties"))
    for blk in np.array_split(np.arange(len(tr)), a.buckets):
        r = tr[blk]
        print("%5d-%-7d %9.0f %11.0f %6.3f %8.4f %8.4f %8.4f %8.4f %6.3f %5.2f" % (
            blk[0], blk[-1], r[:, C["count"]].mean(), r[:, C["live"]].mean(),
            r[:, C["streamed"]].sum() / max(r[:, C["slots"]].sum(), 1), r[:, C["scan_ms"]].mean(),
            r[:, C["replace_ms"]].mean(), r[:, C["select_ms"]].mean(), r[:, C["wall_ms"]].mean(),
            r[:, C["wall_ms"]].sum() / tot_wall, (r[:, C["ties"]] > 1).mean()))
    eng.close()


if __name__ == "__main__":
    main()
