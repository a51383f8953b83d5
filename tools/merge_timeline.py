"""Per-merge kernel timeline of a production C4 train (no events, no probes) from a rocprofv3 kernel trace.

  rocprofv3 --kernel-trace --output-format csv -d D -o run -- python3 tools/merge_timeline.py --run L.json
  python3 tools/merge_timeline.py --analyse D L.json

--run trains C4 twice (warm-up, then the measured train) and writes the measured train's scan log (one
entry per pair-scan launch: 2 x merge index + form, -1 = no-op) and device merge log (ties per merge).
--analyse matches the trace's last pair-scan launches to the scan log; each batch merge's scan is
followed by its zbpe_replace and zbpe_select_next (which starts merge X+1: its duration depends on
whether merge X+1 is a tie). Reports, per merge-index bucket: average scan / replace / select
durations and the gaps between them, with the select split by whether the next merge is tied.
"""
import argparse
import bisect
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DUMP = 0


def run(out, opts):
    sys.path.insert(0, os.path.join(ROOT, "zig-bpe_amd"))
    import zbpe

    e = zbpe.Engine(0)
    e.upload(zbpe.synth_corpus("words_utf8", 0x5EED0004, 1 << 30, threads=16))
    for kv in opts:
        k, v = kv.split("=")
        e.set_option(k, int(v))
    e.train_resident(32000)
    m, c, st = e.train_resident(32000)
    log = e.merge_log()
    json.dump({"scan_log": e.scan_log().tolist(), "ties": log[:, 3].tolist(), "count": log[:, 1].tolist(),
               "live": log[:, 2].tolist(), "halts": e.halt_log().tolist(), "total_s": st.total_s},
              open(out, "w"))
    print(f"{len(m)} merges, {st.total_s:.3f} s")
    e.close()


def analyse(d, logp):
    files = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    if not files:
        sys.exit(f"no kernel trace under {d}")
    ks = []
    for p in files:
        with open(p) as f:
            for r in csv.DictReader(f):
                ks.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r.get("Kernel_Name", "")))
    ks.sort()
    L = json.load(open(logp))
    slog, ties = L["scan_log"], L["ties"]
    scans = [i for i, k in enumerate(ks) if "zbpe_scan_pairs_t" in k[2]]
    if len(scans) < len(slog):
        sys.exit(f"{len(scans)} scans in the trace, {len(slog)} in the log")
    scans = scans[len(scans) - len(slog):]
    buckets = [(0, 100), (100, 500), (500, 2000), (2000, 8000), (8000, 20000), (20000, 1 << 30)]
    dens_acc = {}
    acc = {b: {} for b in buckets}

    def add(b, k, v):
        a = acc[b].setdefault(k, [0.0, 0, []])
        a[0] += v
        a[1] += 1
        a[2].append(v)

    for j, x in enumerate(slog):
        if x < 0:
            continue
        mi, form = x >> 1, x & 1
        i = scans[j]
        if i + 3 >= len(ks):
            continue
        s, r, sel, nxt = ks[i], ks[i + 1], ks[i + 2], ks[i + 3]
        if "zbpe_replace" not in r[2] or "zbpe_select_next" not in sel[2]:
            continue
        b = next(bb for bb in buckets if bb[0] <= mi < bb[1])
        add(b, "scan_" + ("list" if form else "stream"), (s[1] - s[0]) / 1e3)
        if not form and "live" in L:  # stream form: by occurrence density (count / live tokens)
            dens = L["count"][mi] / max(1, L["live"][mi])
            db = next(x for x in (0.0005, 0.002, 0.005, 0.01, 0.02, 1.0) if dens <= x)
            a = dens_acc.setdefault(db, [0.0, 0.0, 0])
            a[0] += (s[1] - s[0])
            a[1] += 2.0 * L["live"][mi]
            a[2] += 1
        add(b, "gap_scan_replace", (r[0] - s[1]) / 1e3)
        add(b, "replace", (r[1] - r[0]) / 1e3)
        add(b, "gap_replace_select", (sel[0] - r[1]) / 1e3)
        nt = mi + 1 < len(ties) and ties[mi + 1] > 1
        add(b, "select_next_tied" if nt else "select_next_untied", (sel[1] - sel[0]) / 1e3)
        if "zbpe_scan_pairs_t" in nxt[2]:
            add(b, "gap_select_scan", (nxt[0] - sel[1]) / 1e3)
            add(b, "merge_total", (nxt[0] - s[0]) / 1e3)
    # wall time per bucket from the trace: the first scan launch of the bucket's first merge to the next bucket's
    # (everything in between: kernels, gaps, batch-boundary syncs, halts and their host path, compactions)
    first = {}
    for j, x in enumerate(slog):
        if x >= 0:
            first.setdefault(x >> 1, ks[scans[j]][0])
    wall = {}
    for b in buckets:
        lo = min((m for m in first if m >= b[0]), default=None)
        hi = min((m for m in first if m >= b[1]), default=None)
        if lo is None:
            continue
        t1 = first[hi] if hi is not None else ks[-1][1]
        n = (hi if hi is not None else len(ties)) - lo
        wall[b] = ((t1 - first[lo]) / 1e6, n)  # (trace timestamps in ns)
    # halted batches: reason -> count and host-path microseconds, by bucket
    names = {2: "hot_list_rebuild", 3: "zig_capacity", 4: "undecided_tie", 5: "self_pair", 6: "arena"}
    halts = {b: {} for b in buckets}
    for x, reason, us in L.get("halts", []):
        b = next(bb for bb in buckets if bb[0] <= x - 256 < bb[1])
        h = halts[b].setdefault(names.get(reason, str(reason)), [0, 0.0])
        h[0] += 1
        h[1] += us
    # what a halt's host path runs: the kernels between the previous merge's select and the next merge's first
    # scan (the halted merge on the synchronous path, compactions, rebuilds), by reason: window wall and kernel time
    scan_at = {}
    for j, x in enumerate(slog):
        if x >= 0:
            scan_at.setdefault(x >> 1, scans[j])
    hwin = {}
    for x, reason, us in L.get("halts", []):
        m = x - 256
        if m - 1 not in scan_at or m + 1 not in first:
            continue
        i0 = scan_at[m - 1]
        t_lo = ks[min(i0 + 2, len(ks) - 1)][1]
        t_hi = first[m + 1]
        h = hwin.setdefault(names.get(reason, str(reason)), {"n": 0, "window_us": 0.0, "kernels": {}})
        if DUMP and reason == 5 and m < DUMP:  # the window's kernels: start offset, duration (us)
            seq = [(round((a0 - t_lo) / 1e3, 1), round((a1 - a0) / 1e3, 1), name.split("(")[0].replace("void ", "")[:28])
                   for a0, a1, name in ks[i0 + 3:] if t_lo <= a0 < t_hi]
            print(json.dumps({"halt_merge": m, "host_us": us, "window_us": round((t_hi - t_lo) / 1e3, 1), "kernels": seq}), file=sys.stderr)
        h["n"] += 1
        h["window_us"] += (t_hi - t_lo) / 1e3
        for a0, a1, name in ks[i0 + 3:]:
            if a0 >= t_hi:
                break
            if a0 >= t_lo:
                short = name.split("(")[0].replace("void ", "").replace("zbpe::", "")[:40]
                h["kernels"][short] = h["kernels"].get(short, 0.0) + (a1 - a0) / 1e3
    out = {}
    out["halt_windows"] = {k: {"n": v["n"], "window_us_avg": round(v["window_us"] / v["n"], 1),
                               "kernel_us_avg": {kk: round(vv / v["n"], 1) for kk, vv in sorted(v["kernels"].items(), key=lambda kv: -kv[1])[:8]}}
                           for k, v in hwin.items()}
    for b in buckets:
        key = f"merges [{b[0]}, {b[1] if b[1] < 1 << 30 else 'end'})"
        if b in wall:
            nl = sum(1 for x in slog if x >= 0 and b[0] <= (x >> 1) < b[1])  # scan launches (a multi-merge round: one)
            out[key + " wall"] = {"ms": round(wall[b][0], 2), "merges": wall[b][1], "us_per_merge": round(wall[b][0] * 1e3 / max(1, wall[b][1]), 2),
                                  "scan_launches": nl, "merges_per_launch": round(wall[b][1] / max(1, nl), 3)}
        out[key + " halts"] = {k: {"n": v[0], "host_us_avg": round(v[1] / v[0], 1), "host_ms": round(v[1] / 1e3, 2)}
                               for k, v in sorted(halts[b].items())}
    for b in buckets:
        out[f"merges [{b[0]}, {b[1] if b[1] < 1 << 30 else 'end'})"] = {
            k: {"avg_us": round(v[0] / v[1], 2), "p50_us": round(sorted(v[2])[len(v[2]) // 2], 2), "n": v[1]}
            for k, v in sorted(acc[b].items())}
    # kernel time of the measured train by kernel (from its first pair scan to the end of the trace)
    t0 = ks[scans[0]][0]
    tot = {}
    for a0, a1, name in ks:
        if a0 >= t0:
            short = name.split("(")[0].replace("void ", "").replace("zbpe::", "")[:40]
            tot[short] = tot.get(short, 0.0) + (a1 - a0) / 1e6
    out["kernel_ms_measured_train"] = {k: round(v, 2) for k, v in sorted(tot.items(), key=lambda kv: -kv[1])[:14]}
    out["stream_scans_by_density"] = {
        f"count/live <= {k}": {"launches": v[2], "avg_us": round(v[0] / v[2] / 1e3, 2), "alg_GBps": round(v[1] / v[0], 1)}
        for k, v in sorted(dens_acc.items())}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    p = argparse.ArgumentParser()
    p.add_argument("--run", default="")
    p.add_argument("--analyse", nargs=2, default=None)
    p.add_argument("--opt", action="append", default=[], help="engine option k=v")
    p.add_argument("--dump-self", type=int, default=0, help="print the kernels of self-pair halts below this merge to stderr")
    a = p.parse_args()
    DUMP = a.dump_self
    if a.run:
        run(a.run, a.opt)
    if a.analyse:
        analyse(*a.analyse)
