"""Single-GPU trains under contention: `procs` processes share cuda:0, each training one case of tests/test_dist.py
(world 1, no collective) `reps` times and comparing every run with the oracle. Prints the failures per process.
  python3 tools/contention_check.py --case 10 --procs 8 --reps 6 [--opt k=v ...]"""
import argparse
import json
import multiprocessing as mp
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "zig-bpe_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)


def worker(i, case, reps, opts, ref, q):
    import zbpe
    import test_dist as T

    text = T.case_text(case)
    fails = []
    e = zbpe.Engine(0)
    for k, v in opts.items():
        e.set_option(k, v)
    for r in range(reps):
        try:
            m, c, st = e.train(text, case["vocab"])
            if m.tolist() != ref[0] or c.tolist() != ref[1]:
                fails.append(f"run {r}: merges differ")
        except zbpe.ZbpeError as x:
            fails.append(f"run {r}: {str(x)[-200:]}")
    e.close()
    q.put((i, fails))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--case", type=int, default=10)
    ap.add_argument("--procs", type=int, default=8)
    ap.add_argument("--reps", type=int, default=6)
    ap.add_argument("--opt", action="append", default=[])
    a = ap.parse_args()
    import oracle as O
    import test_dist as T

    case = dict(T.CASES[a.case])
    opts = dict(case.get("options", {}))
    opts.pop("replicate_late", None)
    for kv in a.opt:
        k, v = kv.split("=")
        opts[k] = int(v)
    r = O.train(T.case_text(case), case["vocab"])
    ref = (r.merges.tolist(), r.counts.tolist())
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=worker, args=(i, case, a.reps, opts, ref, q)) for i in range(a.procs)]
    for p in ps:
        p.start()
    out = dict(q.get(timeout=600) for _ in ps)
    for p in ps:
        p.join(timeout=60)
    nf = sum(len(v) for v in out.values())
    print(json.dumps({"case": a.case, "opts": opts, "procs": a.procs, "reps": a.reps, "failures": nf,
                      "first": next((v[0] for v in out.values() if v), None)}))


if __name__ == "__main__":
    main()
