"""The exact-tie window inside a C4 train (options exact_ties_from / exact_ties_to): every tie decision of the window
taken by both the device's cluster test and the exact Zig-map emulation; prints per round_k the error or the tie
cross-checks and whether the merges equal the full C4 golden. GPU box:
  python3 tools/exact_window_check.py [--from 25000] [--to 25070] [--k 5 --k 1]"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "zig-bpe_amd"))


def main():
    import zbpe

    p = argparse.ArgumentParser()
    p.add_argument("--from", dest="lo", type=int, default=25000)
    p.add_argument("--to", dest="hi", type=int, default=25070)
    p.add_argument("--k", action="append", type=int, default=[])
    p.add_argument("--checks", type=int, default=0, help="option batch_checks: recount after every batch past this merge")
    a = p.parse_args()
    g = json.load(open(os.path.join(ROOT, "tests", "golden", "large_c4_words_utf8_1GiB_v32000.json")))
    text = zbpe.synth_corpus("words_utf8", 0x5EED0004, 1 << 30, threads=16)
    e = zbpe.Engine(0)
    e.upload(text)
    del text
    for k in a.k or [5, 1]:
        e.set_option("round_k", k)
        e.set_option("exact_ties_from", a.lo)
        e.set_option("exact_ties_to", a.hi)
        e.set_option("batch_checks", a.checks)
        r = {"round_k": k}
        try:
            m, c, st = e.train_resident(32000)
            K = g["n_merges"]
            r.update(crosschecks=st.tie_crosschecks, fallbacks=st.tie_fallbacks,
                     merges_equal=m[:K].tolist() == g["merges"], counts_equal=c[:K].tolist() == g["counts"])
        except zbpe.ZbpeError as x:
            r["error"] = str(x)
        print(json.dumps(r), flush=True)
    e.close()


if __name__ == "__main__":
    main()
