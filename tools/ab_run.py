"""A/B of engine options on one C4 train each: python tools/ab_run.py --cfg "merge_timing=1" --cfg "merge_timing=8,merge_batch=64"
Every configuration trains the same resident corpus (one warm-up train first); prints merges/s per config
and checks that every configuration produced the same merges as the first."""
import argparse
import json
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
    p.add_argument("--cfg", action="append", default=[])
    p.add_argument("--reps", type=int, default=1)
    a = p.parse_args()
    cfgs = a.cfg or [""]
    eng = zbpe.Engine(0)
    eng.upload(zbpe.synth_corpus("words_utf8", a.seed, a.n_bytes, threads=16))
    ref, _, _ = eng.train_resident(a.vocab)
    for cfg in cfgs:
        e = zbpe.Engine(0)
        e.upload(zbpe.synth_corpus("words_utf8", a.seed, a.n_bytes, threads=16))
        for kv in filter(None, cfg.split(",")):
            k, v = kv.split("=")
            e.set_option(k, int(v))
        best = 1e9
        for _ in range(a.reps + 1):
            t = time.perf_counter()
            m, c, st = e.train_resident(a.vocab)
            best = min(best, time.perf_counter() - t)
        same = bool(np.array_equal(m, ref))
        print(json.dumps({"cfg": cfg, "merges_per_s": len(m) / best, "s": best, "same_merges": same,
                          "scan_s": st.scan_kernel_s,
                          "scan_alg_GBps": st.scan_timed_alg_bytes / max(st.scan_kernel_s, 1e-12) / 1e9, "ev_count_s": st.count_pairs_s, "ev_select_s": st.sort_pairs_s,
                          "ev_replace_s": st.replace_pair_s, "list_scans": st.list_scans,
                          "pair_selects": getattr(st, "pair_selects", 0), "round_merges": getattr(st, "round_merges", 0), "tie_iterations": st.tie_iterations}), flush=True)
        e.close()
    eng.close()


if __name__ == "__main__":
    main()
