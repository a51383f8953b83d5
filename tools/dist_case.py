"""Run one multi-rank case of tests/test_dist.py (ranks sharing cuda:0, gloo host collectives) and report per rank:
error text or the first merge that differs from the oracle, and the sharding statistics.

  python3 tools/dist_case.py --world 8 --case 13 [--opt key=value ...]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "zig-bpe_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--case", type=int, default=13)
    ap.add_argument("--opt", action="append", default=[])
    a = ap.parse_args()
    import oracle as O
    import test_dist as T
    from dist_worker import run, train_worker

    case = dict(T.CASES[a.case])
    case["options"] = dict(case.get("options", {}))
    for kv in a.opt:
        k, v = kv.split("=")
        case["options"][k] = int(v)
    text = T.case_text(case)
    ref = O.train(text, case["vocab"])
    rm, rc = ref.merges.tolist(), ref.counts.tolist()
    try:
        out = run(train_worker, a.world, case)
    except RuntimeError as e:
        print(json.dumps({"world": a.world, "case": a.case, "options": case["options"], "error": str(e).splitlines()[-1]}))
        return 0  # (reported; a non-zero exit is left to crashes and time limits)
    res = {"world": a.world, "case": a.case, "options": case["options"], "oracle_pair_tokens": int(ref.stats.pair_tokens),
           "sum_tokens": int(out[0][3]["sum_tokens"]), "final_tokens": int(out[0][3]["final_tokens"]), "oracle_final": len(ref.tokens)}
    for r in range(a.world):
        _, m, c, st = out[r][:4]
        diff = next((i for i in range(max(len(m), len(rm))) if i >= len(m) or i >= len(rm) or m[i] != rm[i] or c[i] != rc[i]), None)
        res[f"rank{r}"] = {"first_diff": diff, "merges": len(m), "sharded_merges": st["sharded_merges"],
                           "replications": st["replications"], "compactions": st["compactions"],
                           "round_merges": st.get("round_merges"), "self_pair_merges": st.get("self_pair_merges")}
    print(json.dumps(res))
    return 0


if __name__ == "__main__":
    sys.exit(main())
