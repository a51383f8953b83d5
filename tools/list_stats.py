"""Occurrence-list walk statistics of one C4 train (zbpe_merge_log): per merge bucket, the pair count,
the walked list length and the live occurrences of the list's token (the useful entries).

  python tools/list_stats.py [--n-bytes B] [--vocab V] [--buckets 12]
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "zig-bpe_amd"))
import zbpe  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--n-bytes", type=int, default=1 << 30)
    p.add_argument("--vocab", type=int, default=32000)
    p.add_argument("--seed", type=int, default=0x5EED0004)
    p.add_argument("--buckets", type=int, default=12)
    a = p.parse_args()
    e = zbpe.Engine(0)
    e.upload(zbpe.synth_corpus("words_utf8", a.seed, a.n_bytes, threads=16))
    m, c, st = e.train_resident(a.vocab)
    L = e.merge_log().astype(np.float64)
    C = {k: i for i, k in enumerate(zbpe.MERGE_LOG_COLUMNS)}
    print(f"{len(m)} merges, {int(st.list_scans)} list scans, {int(st.compactions)} compactions, {int(st.list_builds)} list builds")
    print("%-13s %9s %7s %10s %10s %9s" % ("merges", "count", "lists", "walked", "key_live", "walk/cnt"))
    for blk in np.array_split(np.arange(len(L)), a.buckets):
        r = L[blk]
        ls = r[r[:, C["list_scan"]] > 0]
        if len(ls) == 0:
            print("%5d-%-7d %9.0f %7d" % (blk[0], blk[-1], r[:, C["count"]].mean(), 0))
            continue
        print("%5d-%-7d %9.0f %7d %10.0f %10.0f %9.1f" % (blk[0], blk[-1], r[:, C["count"]].mean(), len(ls),
                                                        ls[:, C["list_len"]].mean(), ls[:, C["key_live"]].mean(),
                                                        (ls[:, C["list_len"]] / np.maximum(ls[:, C["count"]], 1)).mean()))
    e.close()


if __name__ == "__main__":
    main()
