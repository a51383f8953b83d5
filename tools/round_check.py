"""Multi-merge rounds against the full goldens (C3, C4): every merge, count and per-merge tie count (the device's
merge log) equal the golden's, for each round_k given; prints the first difference, the round statistics and the
train time. GPU box: python tools/round_check.py [--corpus c3|c4] [--k 1 --k 4 ...] [--opt k=v]"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "zig-bpe_amd"))
sys.path.insert(0, ROOT)

CORPORA = {"c3": (0x5EED0003, 64 << 20, 4096, "large_c3_words_utf8_64MiB_v4096.json"),
           "c4": (0x5EED0004, 1 << 30, 32000, "large_c4_words_utf8_1GiB_v32000.json")}


def main():
    import numpy as np
    import zbpe

    p = argparse.ArgumentParser()
    p.add_argument("--corpus", action="append", default=[])
    p.add_argument("--k", action="append", type=int, default=[])
    p.add_argument("--opt", action="append", default=[])
    a = p.parse_args()
    for c in a.corpus or ["c3", "c4"]:
        seed, n, vocab, gname = CORPORA[c]
        g = json.load(open(os.path.join(ROOT, "tests", "golden", gname)))
        text = zbpe.synth_corpus("words_utf8", seed, n, threads=16)
        for k in a.k or [1, 4]:
            e = zbpe.Engine(0)
            e.upload(text)
            e.set_option("round_k", k)
            for kv in a.opt:
                kk, vv = kv.split("=")
                e.set_option(kk, int(vv))
            e.train_resident(vocab)  # warm-up
            t = time.perf_counter()
            m, cnt, st = e.train_resident(vocab)
            dt = time.perf_counter() - t
            log = e.merge_log()
            ties = log[:, 3].astype(int).tolist()
            mm = m.astype(int).tolist()
            first = next((i for i in range(len(mm)) if mm[i] != g["merges"][i] or int(cnt[i]) != g["counts"][i]), None)
            tfirst = next((i for i in range(len(ties)) if ties[i] and ties[i] != g["ties"][i]), None)
            zero = sum(1 for t_ in ties if t_ == 0)
            out = {"corpus": c, "round_k": k, "merges": len(mm), "first_merge_diff": first, "first_tie_diff": tfirst,
                   "log_rows_zero": zero, "round_merges": st.round_merges, "pair_selects": st.pair_selects,
                   "tie_iterations": st.tie_iterations, "golden_ties": sum(t_ > 1 for t_ in g["ties"]),
                   "mismatches": e.verify_counts(), "train_s": round(dt, 4), "merges_per_s": round(len(mm) / dt, 1)}
            if first is not None:
                out["diff"] = {"at": first, "got": [mm[first], int(cnt[first])], "want": [g["merges"][first], g["counts"][first]]}
            if tfirst is not None:
                out["tie_diff"] = {"at": tfirst, "got": ties[tfirst], "want": g["ties"][tfirst], "merge": mm[tfirst]}
            print(json.dumps(out), flush=True)
            e.close()


if __name__ == "__main__":
    main()
