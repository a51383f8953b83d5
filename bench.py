"""Benchmark: BPE training throughput (merges/s) on the MI355X, BASELINE.json config C4:
a 1 GiB synthetic corpus, vocab_size 32000 (31,744 merges), token stream sharded over N GPUs.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--n-bytes B] [--vocab V]
  N>1: python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...

A step = one complete BasicTokenizer.train() over the whole corpus (all merges), starting from
the corpus bytes already resident in HBM (zbpe_upload is outside the timed region).
Prints ONE JSON line on rank 0 (the driver's contract) with `roofline` (dominant kernel:
zbpe_scan_pairs_t, stream form, HBM-read bound) and `cpu_baseline` (the oracle, timed on this host).

After the K timed steps, one untimed *probe* train runs with HIP events around every merge of every
batch that streams the token stream (option timing_full): `roofline` comes from it, so it covers
nearly every stream-form scan launch, not a 1-in-8 sample (events add gaps, which is why the timed
steps only sample). --scan-log-out writes the probe train's scan log, so a rocprofv3 kernel trace of
this command can be matched launch by launch (tools/scan_forms.py, tools/pmc_traffic.py).
"""
from __future__ import annotations

import argparse
import json
import os
import platform
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "zig-bpe_amd"))

# tools/pmc_traffic.py output: this round's PMC passes when present, else the last round's
PMC_TRAFFIC = next((p for p in (os.path.join(ROOT, "profiles", f"r0{r}_c4_pmc_traffic.json") for r in (6, 5, 4, 3, 2))
                    if os.path.exists(p)), os.path.join(ROOT, "profiles", "r02_c4_pmc_traffic.json"))
HBM_PEAK_GBPS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec (6.29 TB/s measured copy)
C4_SEED = 0x5EED0004
LIST_ENTRY_BYTES = 4 + 16  # a list scan reads the entry's list word and its 16-B stream vector


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=2)
    p.add_argument("--warmup", type=int, default=1)
    p.add_argument("--n-bytes", type=int, default=1 << 30)
    p.add_argument("--vocab", type=int, default=32000)
    p.add_argument("--kind", default="words_utf8")
    p.add_argument("--seed", type=int, default=C4_SEED)
    p.add_argument("--cpu-late-merge", type=int, default=20000,
                   help="cpu_baseline: the late sample is one reference iteration on the GPU's stream after this many merges")
    p.add_argument("--no-cpu", action="store_true")
    p.add_argument("--no-probe", action="store_true", help="skip the roofline probe train")
    p.add_argument("--stats-out", default="")
    p.add_argument("--scan-log-out", default="",
                   help="write the probe train's per-launch scan log + per-merge live tokens (tools/pmc_traffic.py, tools/scan_forms.py)")
    p.add_argument("--share-gpu", action="store_true",
                   help="all ranks on cuda:0 with host (gloo) collectives -- rehearses N>1 on one GPU")
    p.add_argument("--no-extra", action="store_true",
                   help="skip the other BASELINE configs (C1/C2 CPU+GPU, C3 train, C5 encode) and the incremental CPU model")
    p.add_argument("--inc-merges", type=int, default=4,
                   help="cpu_incremental: merges of C4 timed with tests/model/inc_model.cpp")
    return p.parse_args()


def cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or "unknown"


def cpu_baseline(eng, text: bytes, vocab: int, live, late_k: int):
    """The oracle (single-threaded C restatement of basic_tokenizer.zig, gcc -O3) timed on this host for
    ONE reference loop iteration (generateCodePointPairs + countCodePointPairs + sortCodePointPairs,
    literally: materialised pairs, Zig map, stable sort) at two points of the C4 run:
      early: the full 1 GiB initial stream (t = 0; few distinct pairs, the map stays in cache),
      late:  the GPU's own stream after `late_k` merges (zbpe_tokens; ~5e7 distinct pairs, cache-miss bound).
    Replace is O(n) and omitted (it is cheaper than the count). Every merge t costs n_t x ns_per_token(t);
    ns_per_token is interpolated linearly in t between the two samples and held beyond them; the
    GPU run's measured n_t trajectory (`live`) prices the whole job (an extrapolation, labelled so)."""
    import numpy as np

    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle

    tok0 = np.frombuffer(text, np.uint8).astype(np.uint16)
    r0 = oracle.step(tok0, literal=True)
    del tok0
    m, _, _ = eng.train_resident(min(vocab, 256 + late_k))
    late_k = len(m)
    tokl = eng.tokens()
    r1 = oracle.step(tokl, literal=True)
    ns0 = r0.stats.total_s / max(r0.stats.pair_tokens, 1) * 1e9
    ns1 = r1.stats.total_s / max(r1.stats.pair_tokens, 1) * 1e9
    t = np.arange(len(live), dtype=np.float64)
    ns = np.where(t >= late_k, ns1, ns0 + (ns1 - ns0) * t / max(late_k, 1))
    full_s = float(np.sum(np.asarray(live, dtype=np.float64) * ns) * 1e-9)
    merges = len(live)
    return {
        "value": merges / full_s if full_s > 0 else None,
        "unit": "merges/s",
        "cores": 1,
        "kind": "port",
        "cpu_model": cpu_model(),
        "nproc": os.cpu_count(),
        "sample": (f"oracle (C restatement of basic_tokenizer.zig:183-204, gcc -O3, 1 thread) timed for one literal loop "
                   f"iteration at merge 0 on the full {len(text)}-B stream ({r0.stats.total_s:.2f} s, "
                   f"{r0.distinct} distinct pairs, {ns0:.2f} ns/token) and at merge {late_k} on the GPU's stream "
                   f"({len(tokl)} tokens, {r1.distinct} distinct pairs, {r1.stats.total_s:.2f} s, {ns1:.2f} ns/token); "
                   f"the {merges} merges priced over the GPU run's n_t trajectory (sum {int(np.sum(live))} tokens, "
                   f"ns/token interpolated by merge index) -> {full_s / 3600:.1f} h (extrapolated)"),
        "sample_seconds": r0.stats.total_s + r1.stats.total_s,
        "ns_per_token_early": ns0,
        "ns_per_token_late": ns1,
        "late_merge": late_k,
        "oracle_agrees_with_gpu": None,  # filled by the caller
        "extrapolated_full_job_s": full_s,
        "_pairs": (r0.pair, r1.pair),
    }


def cpu_incremental(text: bytes, gpu_merges, k: int):
    """Algorithm-matched CPU figure: tests/model/inc_model.cpp (the device's incremental counting, one
    core, g++ -O3; a pass over the stream per merge finds the occurrences) on the C4 corpus for the
    first k merges, next to the literal port's per-merge cost (cpu_baseline)."""
    import subprocess
    import tempfile

    src = os.path.join(ROOT, "tests", "model", "inc_model.cpp")
    with tempfile.TemporaryDirectory() as d:
        exe, corpus = os.path.join(d, "inc_model"), os.path.join(d, "corpus.bin")
        subprocess.run(["g++", "-O3", "-std=c++17", "-o", exe, src], check=True)
        with open(corpus, "wb") as f:
            f.write(text)
        t = time.perf_counter()
        r = subprocess.run([exe, corpus, "32000", "0", str(k)], capture_output=True, text=True, check=True)
        wall = time.perf_counter() - t
    timing = dict(kv.split("=") for kv in r.stderr.split("timing:")[1].split("\n")[0].split())
    merges = [tuple(int(v) for v in line.split(",")) for line in r.stdout.split()]
    agrees = [list(x) for x in merges] == [list(map(int, row)) for row in gpu_merges[: len(merges)]]
    init_s, merges_s = float(timing["init_s"]), float(timing["merges_s"])
    return {"value": len(merges) / merges_s if merges_s > 0 else None, "unit": "merges/s", "cores": 1,
            "kind": "incremental model (tests/model/inc_model.cpp, g++ -O3)", "merges": len(merges),
            "init_s": init_s, "merges_s": merges_s, "wall_s": wall, "agrees_with_gpu": bool(agrees),
            "sample": f"the first {len(merges)} merges of C4 ({len(text)} B): incremental counts, one stream pass per merge"}


def histogram_roofline(eng, late: int, reps: int = 5):
    """The north-star's full pair-histogram kernel (zbpe_pair_hist_bytes at t = 0, zbpe_pair_hist later: every adjacent pair of the stream,
    LDS-staged per workgroup; the recount behind verify_counts), timed with HIP events at t = 0 (the
    widened 1 GiB stream, ~3.6e3 distinct pairs) and after `late` merges (~5e7 distinct pairs: most pairs
    miss the LDS tables and pay a global lookup). Algorithmic bytes: 2 B per token."""
    out = {}
    for name, v in (("t0", 256), (f"after_{late}", 256 + late)):
        eng.train_resident(v)
        r = eng.bench_recount(reps)
        # at t = 0 every token is a byte: the engine runs zbpe_pair_hist_bytes (all 65,536 byte pairs in 16-bit
        # LDS bins, option dense_hist); later the hashed zbpe_pair_hist
        kern = "zbpe_pair_hist_bytes" if v == 256 else "zbpe_pair_hist"
        out[name] = {"kernel": kern, "bound": "hbm", "achieved": r["GBps"], "peak": HBM_PEAK_GBPS,
                     "unit": "GB/s", "frac": r["GBps"] / HBM_PEAK_GBPS, "avg_launch_us": r["us"], "tokens": r["tokens"],
                     "alg_bytes_per_launch": 2 * r["tokens"], "counts_match_incremental": r["mismatches"] == 0}
    return out


def extra_configs(zbpe, eng, c4_merges, args):
    """The other BASELINE.json configs, under the same clock (rank 0, one GPU):
      c1: taylorswift.txt, V=300 -- the oracle (CPU, full run) and the GPU, merges compared
      c2: 1 MiB synthetic ASCII, V=512 -- the same
      c3: 64 MiB UTF-8 synthetic, V=4096 -- GPU merges/s and the stream-form scan GB/s (its 128 MiB u16
          stream fits the 256 MiB Infinity Cache: L3-resident, not an HBM figure)
      c5: encode 100 M chars with the C4 merges -- chars/s (host buffers in and out, PCIe included), and
          a 200 kB prefix against the oracle's encode"""
    import gzip

    import numpy as np

    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle

    out = {}
    with gzip.open(os.path.join(ROOT, "tests", "golden", "c1_taylorswift.txt.gz"), "rb") as f:
        c1 = f.read()
    c2 = zbpe.synth_corpus("words", 0x5EED0002, 1 << 20)
    for name, text, vocab in (("c1", c1, 300), ("c2", c2, 512)):
        t = time.perf_counter()
        ref = oracle.train(text, vocab)
        cpu_s = time.perf_counter() - t
        eng.train(text, vocab)  # warm
        t = time.perf_counter()
        m, c, st = eng.train(text, vocab)
        gpu_s = time.perf_counter() - t
        out[name] = {"bytes": len(text), "vocab_size": vocab, "merges": int(len(m)),
                     "cpu_oracle_s": cpu_s, "gpu_train_s": gpu_s,
                     "bit_exact": bool(np.array_equal(m, ref.merges) and np.array_equal(c, ref.counts)),
                     "note": "gpu_train_s: zbpe_train with the host buffer (upload included); cpu: the oracle, 1 thread"}
    c3 = zbpe.synth_corpus("words_utf8", 0x5EED0003, 64 << 20, threads=16)
    eng.upload(c3)
    eng.train_resident(4096)
    times = []
    for _ in range(3):
        t = time.perf_counter()
        m3, c3c, st3 = eng.train_resident(4096)
        times.append(time.perf_counter() - t)
    eng.set_option("timing_full", 1)
    _, _, sp = eng.train_resident(4096)
    eng.set_option("timing_full", 0)
    gbps = sp.scan_timed_alg_bytes / sp.scan_kernel_s / 1e9 if sp.scan_kernel_s > 0 else 0.0
    out["c3"] = {"bytes": len(c3), "vocab_size": 4096, "merges": int(len(m3)), "value": len(m3) / min(times),
                 "unit": "merges/s", "best_s": min(times),
                 "stream_scan_GBps": gbps, "stream_scan_launches_timed": int(sp.scan_timed_launches),
                 "stream_scan_note": "L3-resident: the 128 MiB u16 stream fits the 256 MiB Infinity Cache",
                 "ties": int(st3.tie_iterations)}
    del c3
    c5 = zbpe.synth_corpus("words_utf8", 0x5EED0005, 100_000_000, threads=16)
    eng.encode(c4_merges, c5[: 1 << 20])  # warm
    times = []
    enc = None
    for _ in range(2):
        t = time.perf_counter()
        enc = eng.encode(c4_merges, c5)
        times.append(time.perf_counter() - t)
    pre = c5[:200_000]
    out["c5"] = {"chars": len(c5), "merges": int(len(c4_merges)), "value": len(c5) / min(times), "unit": "chars/s",
                 "best_s": min(times), "tokens_out": int(len(enc)),
                 "prefix_equals_oracle": bool(np.array_equal(eng.encode(c4_merges, pre), oracle.encode(c4_merges, pre))),
                 "prefix_bytes": len(pre), "note": "zbpe_encode with host buffers in and out (PCIe included)"}
    return out


def probe_roofline(eng, vocab: int, scan_log_out: str):
    """One untimed train with events around (nearly) every stream-form scan: the roofline of the
    stream form from HIP events on the engine's stream, plus the list form's rate."""
    import numpy as np
    import zbpe

    eng.set_option("timing_full", 1)
    eng.set_option("merge_timing", 1)  # every merge: the list form's figure covers all its launches, late ones too
    eng.set_option("trace", 1)
    m, c, st = eng.train_resident(vocab)
    eng.set_option("timing_full", 0)
    eng.set_option("merge_timing", 8)
    tr = eng.trace()
    eng.set_option("trace", 0)
    C = {k: i for i, k in enumerate(zbpe.TRACE_COLUMNS)}
    log = eng.scan_log()
    live = tr[:, C["live"]].astype(np.int64)
    if scan_log_out:
        with open(scan_log_out, "w") as f:
            json.dump({"scan_log": log.tolist(), "live": live.tolist()}, f)
    # list form: the timed list-scan merges (scan_ms > 0; the walked list length is in `streamed`)
    forms = {}
    for e in log:
        if e >= 0:
            forms[int(e) >> 1] = int(e) & 1
    lms, lent = 0.0, 0.0
    nl = 0
    for i, r in enumerate(tr):
        if forms.get(i) == 1 and r[C["scan_ms"]] > 0 and r[C["streamed"]] > 0:
            lms += float(r[C["scan_ms"]])
            lent += float(r[C["streamed"]])
            nl += 1
    achieved = st.scan_timed_alg_bytes / st.scan_kernel_s / 1e9 if st.scan_kernel_s > 0 else 0.0
    n_stream = int(np.sum(np.array([f == 0 for f in forms.values()])))
    return {
        "achieved": achieved,
        "timed_launches": int(st.scan_timed_launches),
        "stream_launches": n_stream,
        "avg_launch_us": st.scan_kernel_s / max(st.scan_timed_launches, 1) * 1e6,
        "alg_bytes_per_launch": st.scan_timed_alg_bytes / max(st.scan_timed_launches, 1),
        "list_form": {"timed_launches": nl, "avg_launch_us": lms / max(nl, 1) * 1e3,
                      "avg_entries": lent / max(nl, 1),
                      "GBps": lent * LIST_ENTRY_BYTES / max(lms * 1e-3, 1e-12) / 1e9,
                      "note": "every list-form launch of the probe train (HIP events around each merge's scan: ~1 us of "
                              "event gap each); bytes = 4 B list word + 16 B stream vector per walked entry; "
                              "latency-bound (a chain of dependent loads and atomics per entry), not bandwidth-bound"},
        "merges": m, "counts": c, "live": live,
    }


def make_engine(zbpe, share_gpu: bool, rank: int, world: int, local_rank: int, dist):
    """One engine per rank (one process per GPU). N>1: rank 0's RCCL unique id is broadcast over the
    gloo group and every rank joins the RCCL communicator on its own GPU; if RCCL cannot initialise,
    the exchange falls back to host (gloo) collectives and the GPU compute path stays. share_gpu: all
    ranks on cuda:0 with host collectives (rehearses N>1 on one GPU). -> (engine, comm backend name)."""
    if world == 1:
        return zbpe.Engine(0), "none"
    if share_gpu:
        return (zbpe.Engine(0, rank=rank, world=world, collective=zbpe.torch_collective(rank, world)),
                "gloo (host collectives, ranks share cuda:0)")
    uid = [zbpe.comm_unique_id() if rank == 0 else None]
    dist.broadcast_object_list(uid, src=0)
    try:
        return zbpe.Engine(local_rank, rank=rank, world=world, unique_id=uid[0]), "rccl"
    except zbpe.ZbpeError as e:  # keep the GPU compute path; move only the exchange to gloo
        sys.stderr.write(f"rank {rank}: RCCL init failed ({e}); using host (gloo) collectives\n")
        return (zbpe.Engine(local_rank, rank=rank, world=world, collective=zbpe.torch_collective(rank, world)),
                "gloo (host collectives; RCCL init failed)")


def main():
    args = parse()
    import numpy as np
    import zbpe

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus != world:
        world = args.gpus if world == 1 and args.gpus == 1 else world
    dist = None
    if world > 1:
        import torch.distributed as dist  # noqa: F811

        dist.init_process_group("gloo", init_method="env://")
    eng, comm_backend = make_engine(zbpe, args.share_gpu, rank, world, local_rank, dist)

    t0 = time.time()
    text = zbpe.synth_corpus(args.kind, args.seed, args.n_bytes, threads=16)
    gen_s = time.time() - t0
    t_up = time.perf_counter()
    eng.upload(text)  # HBM-resident before timing (this rank's shard)
    upload_s = time.perf_counter() - t_up

    def barrier():
        if dist is not None:
            dist.barrier()

    for _ in range(args.warmup):
        eng.train_resident(args.vocab)
    times = []
    last = None
    for _ in range(args.steps):
        barrier()
        t = time.perf_counter()
        m, c, st = eng.train_resident(args.vocab)
        dt = time.perf_counter() - t
        barrier()
        times.append(dt)
        last = (m, c, st)
    total = sum(times)
    if dist is not None:
        import torch

        tt = torch.tensor([total], dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        total = float(tt.item())
    m, c, st = last
    merges = len(m)
    value = merges * args.steps / total
    # SURVEY 8(d) prices merges/s with the H2D copy of the corpus: upload it again (timed, same host buffer) and
    # report that rate beside `value` (which starts from HBM-resident bytes)
    barrier()
    t_up = time.perf_counter()
    eng.upload(text)
    upload2_s = time.perf_counter() - t_up
    if dist is not None:
        import torch

        ut = torch.tensor([upload2_s], dtype=torch.float64)
        dist.all_reduce(ut, op=dist.ReduceOp.MAX)
        upload2_s = float(ut.item())
    sampled = st.scan_timed_alg_bytes / st.scan_kernel_s / 1e9 if st.scan_kernel_s > 0 else 0.0
    probe = None if args.no_probe else probe_roofline(eng, args.vocab, args.scan_log_out if rank == 0 else "")
    if probe is not None and not np.array_equal(probe["merges"], m):
        raise SystemExit("probe train produced different merges than the timed steps")
    achieved = probe["achieved"] if probe else sampled
    traffic, traffic_note = None, "no PMC pass for this configuration"
    if os.path.exists(PMC_TRAFFIC) and args.n_bytes == 1 << 30 and args.vocab == 32000 and world == 1:
        t = json.load(open(PMC_TRAFFIC))["traffic"]["stream"]
        traffic = t["hbm_bytes_per_launch"]
        traffic_note = ("HBM bytes per stream-form scan launch (FETCH_SIZE x2 + WRITE_SIZE, rocprofv3 PMC passes of "
                        "`bench.py --steps 1 --warmup 0 --no-cpu`, %s): %.3g x the algorithmic bytes"
                        % (os.path.relpath(PMC_TRAFFIC, ROOT), t["hbm_over_alg"]))
    if rank == 0:
        stats = {k: v for k, v in st.as_dict().items()}
        res = {
            "metric": "merges/sec (BasicTokenizer.train, 1 GiB corpus, vocab 32000) + pair-count HBM GB/s",
            "value": value,
            "unit": "merges/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": total / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "u16",
            "data": f"synthetic: seeded {args.kind} corpus (seed {args.seed:#x}, Zipf(1.1) pseudo-words, 5% UTF-8 words), "
                    f"{args.n_bytes} bytes; no Wikipedia dump offline",
            "config": {"workload": "C4: train vocab_size=%d on a %d-byte corpus" % (args.vocab, args.n_bytes),
                       "corpus_bytes": args.n_bytes, "vocab_size": args.vocab, "merges": merges,
                       "parallelism": "single GPU" if world == 1 else f"token stream sharded x{world}",
                       "comm": comm_backend},
            "roofline": {
                "kernel": "zbpe_scan_pairs_t (stream form)",
                "bound": "hbm",
                "achieved": achieved,
                "peak": HBM_PEAK_GBPS,
                "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBPS,
                "traffic": traffic,
                "traffic_note": traffic_note,
                "note": ("per GPU (rank 0): achieved = algorithmic bytes (2 B x live tokens, SURVEY.md 8d) of the stream-form "
                         "scan launches timed with HIP events on the engine stream in the probe train / their summed "
                         "durations; %s" % (
                             "%d of %d stream launches timed, %.1f us and %.3g GB per launch on average; the timed steps' "
                             "1-in-8 sample gave %.0f GB/s" % (probe["timed_launches"], probe["stream_launches"],
                                                                probe["avg_launch_us"], probe["alg_bytes_per_launch"] / 1e9,
                                                                sampled) if probe else "timed steps' 1-in-8 sample")),
            },
            "pair_count_GBps": achieved,
            "list_scan": probe["list_form"] if probe else None,
            "time_stats": {k: stats[k] for k in ("count_pairs_s", "sort_pairs_s", "replace_pair_s", "other_s", "total_s")},
            "stats": stats,
            "corpus_gen_s": gen_s,
            "h2d": {"upload_s": upload2_s, "first_upload_s": upload_s,
                    "merges_per_s_incl_upload": merges / (total / args.steps + upload2_s),
                    "note": "zbpe_upload of the corpus bytes from a host buffer (PCIe, pageable memory) timed after the "
                            "steps; merges_per_s_incl_upload = merges / (ms_per_step + upload_s): SURVEY 8(d)'s rate with "
                            "the H2D copy; `value` starts from HBM-resident bytes"},
        }
        if world > 1:
            res["phases"] = {k: stats.get(k) for k in ("sharded_s", "replicate_s", "replicated_s", "comm_s", "sharded_merges")}
        if not args.no_cpu and world == 1 and probe is not None:
            cb = cpu_baseline(eng, text, args.vocab, probe["live"], args.cpu_late_merge)
            p0, p1 = cb.pop("_pairs")
            k = cb["late_merge"]
            cb["oracle_agrees_with_gpu"] = bool(p0 == tuple(int(v) for v in m[0, :2]) and
                                                (k >= len(m) or p1 == tuple(int(v) for v in m[k, :2])))
            res["cpu_baseline"] = cb
            if args.inc_merges > 0:
                res["cpu_incremental"] = cpu_incremental(text, m, args.inc_merges)
        if "cpu_baseline" not in res:  # N > 1 (rank 0 only at N = 1), --no-cpu or --no-probe
            res["cpu_baseline"] = None
        if world == 1 and not args.no_extra:
            res["roofline_pair_histogram"] = histogram_roofline(eng, min(args.cpu_late_merge, merges))
        if world == 1 and not args.no_extra and args.n_bytes == 1 << 30 and args.vocab == 32000:
            res["configs"] = extra_configs(zbpe, eng, m, args)
        if args.stats_out:
            with open(args.stats_out, "w") as f:
                json.dump({"merges": m.tolist(), "counts": c.tolist()}, f)
        print(json.dumps(res), flush=True)
    eng.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
