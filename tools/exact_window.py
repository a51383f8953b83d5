"""Cost of the exact Zig-order tie emulation at scale: one train with the exact-tie window
(options exact_ties_from / exact_ties_to) against one without, same corpus.

  python tools/exact_window.py [--n-bytes B] [--vocab V] [--seed S] --from K0 --to K1 [--opt k=v ...]

Prints the wall of both trains, the ties in the window, how many of them both paths decided
(tie_crosschecks) and the extra seconds per exact tie; checks that both trains give the same merges.
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
    p.add_argument("--seed", type=lambda s: int(s, 0), default=0x5EED0004)
    p.add_argument("--from", dest="k0", type=int, required=True)
    p.add_argument("--to", dest="k1", type=int, required=True)
    p.add_argument("--opt", action="append", default=[])
    a = p.parse_args()
    text = zbpe.synth_corpus("words_utf8", a.seed, a.n_bytes, threads=16)
    eng = zbpe.Engine(0)
    for o in a.opt:
        k, v = o.split("=")
        eng.set_option(k, int(v))
    eng.upload(text)
    t = time.perf_counter()
    m0, c0, st0 = eng.train_resident(a.vocab)
    w0 = time.perf_counter() - t
    print(f"plain: {len(m0)} merges {w0:.3f} s, ties {st0.tie_iterations}, fallbacks {st0.tie_fallbacks}", flush=True)
    eng.set_option("exact_ties_from", a.k0)
    eng.set_option("exact_ties_to", a.k1)
    t = time.perf_counter()
    m1, c1, st1 = eng.train_resident(a.vocab)
    w1 = time.perf_counter() - t
    ties_win = int(st1.tie_fallbacks)
    print(f"exact window [{a.k0}, {a.k1}): {w1:.3f} s, exact ties {ties_win}, crosschecks {st1.tie_crosschecks}, "
          f"extra {(w1 - w0) / max(ties_win, 1):.3f} s per exact tie, live pairs {st1.distinct_pairs}", flush=True)
    assert np.array_equal(m0, m1) and np.array_equal(c0, c1), "exact window changed the merges"
    print("same merges: yes")
    eng.close()


if __name__ == "__main__":
    main()
