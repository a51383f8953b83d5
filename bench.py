"""Benchmark: BPE training throughput (merges/s) on the MI355X, BASELINE.json config C4:
a 1 GiB synthetic corpus, vocab_size 32000 (31,744 merges), token stream sharded over N GPUs.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--n-bytes B] [--vocab V]
  N>1: python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...

A step = one complete BasicTokenizer.train() over the whole corpus (all merges), starting from
the corpus bytes already resident in HBM (zbpe_upload is outside the timed region).
Prints ONE JSON line on rank 0 (the driver's contract) with `roofline` (dominant kernel:
zbpe_scan_pairs, HBM-read bound) and `cpu_baseline` (the oracle, timed on this host).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "zig-bpe_amd"))

PMC_TRAFFIC = os.path.join(ROOT, "profiles", "r01_c4_pmc_traffic.json")  # tools/pmc_traffic.py output
HBM_PEAK_GBPS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec (6.29 TB/s measured copy)
C4_SEED = 0x5EED0004


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=2)
    p.add_argument("--warmup", type=int, default=1)
    p.add_argument("--n-bytes", type=int, default=1 << 30)
    p.add_argument("--vocab", type=int, default=32000)
    p.add_argument("--kind", default="words_utf8")
    p.add_argument("--seed", type=int, default=C4_SEED)
    p.add_argument("--cpu-sample-bytes", type=int, default=128 << 20)
    p.add_argument("--cpu-sample-merges", type=int, default=2)
    p.add_argument("--no-cpu", action="store_true")
    p.add_argument("--stats-out", default="")
    p.add_argument("--scan-log-out", default="",
                   help="write the per-launch scan log + per-merge live tokens of the last step (for tools/pmc_traffic.py)")
    p.add_argument("--share-gpu", action="store_true",
                   help="all ranks on cuda:0 with host (gloo) collectives -- rehearses N>1 on one GPU")
    return p.parse_args()


def cpu_baseline(text: bytes, sample_bytes: int, sample_merges: int, vocab: int, sum_tokens: int, merges: int):
    """Oracle (single-threaded C restatement of basic_tokenizer.zig, -O3) on a bounded sample:
    the first `sample_merges` merges of the first `sample_bytes` bytes. Its cost per merge is
    linear in the stream length (pairs hashed per merge = n_t - 1), so the full job is priced from
    the measured seconds per token x the GPU run's exact trajectory sum_t n_t."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle

    sample = text[:sample_bytes]
    r = oracle.train(sample, min(vocab, 256 + sample_merges))
    st = r.stats
    per_token = st.total_s / max(st.pair_tokens, 1)
    full_s = per_token * sum_tokens
    return {
        "value": merges / full_s if full_s > 0 else None,
        "unit": "merges/s",
        "cores": 1,
        "kind": "port",
        "sample": (f"oracle (C restatement, gcc -O3, 1 thread) trained {len(r.merges)} merges on the first "
                   f"{len(sample)} B of the corpus in {st.total_s:.2f} s ({per_token * 1e9:.2f} ns per stream token per "
                   f"merge); full job extrapolated over the GPU run's sum_t n_t = {sum_tokens} tokens "
                   f"-> {full_s / 3600:.1f} h"),
        "sample_seconds": st.total_s,
        "ns_per_token_merge": per_token * 1e9,
        "extrapolated_full_job_s": full_s,
    }


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
    comm_backend = "none"
    if world > 1:
        import torch.distributed as dist  # noqa: F811

        dist.init_process_group("gloo", init_method="env://")
        if args.share_gpu:
            eng = zbpe.Engine(0, rank=rank, world=world, collective=zbpe.torch_collective(rank, world))
            comm_backend = "gloo (host collectives, ranks share cuda:0)"
        else:
            uid = [zbpe.comm_unique_id() if rank == 0 else None]
            dist.broadcast_object_list(uid, src=0)
            try:
                eng = zbpe.Engine(local_rank, rank=rank, world=world, unique_id=uid[0])
                comm_backend = "rccl"
            except zbpe.ZbpeError as e:  # keep the GPU compute path; move only the exchange to gloo
                sys.stderr.write(f"rank {rank}: RCCL init failed ({e}); using host (gloo) collectives\n")
                eng = zbpe.Engine(local_rank, rank=rank, world=world, collective=zbpe.torch_collective(rank, world))
                comm_backend = "gloo (host collectives; RCCL init failed)"
    else:
        eng = zbpe.Engine(0)

    t0 = time.time()
    text = zbpe.synth_corpus(args.kind, args.seed, args.n_bytes, threads=16)
    gen_s = time.time() - t0
    eng.upload(text)  # HBM-resident before timing (this rank's shard)
    if args.scan_log_out:
        eng.set_option("trace", 1)

    def barrier():
        if dist is not None:
            dist.barrier()

    for _ in range(args.warmup):
        eng.train_resident(args.vocab)
    times = []
    scan_s = alg_bytes = all_alg_bytes = read_bytes = 0.0
    last = None
    for _ in range(args.steps):
        barrier()
        t = time.perf_counter()
        m, c, st = eng.train_resident(args.vocab)
        dt = time.perf_counter() - t
        barrier()
        times.append(dt)
        scan_s += st.scan_kernel_s
        alg_bytes += st.scan_timed_alg_bytes
        all_alg_bytes += st.scan_alg_bytes
        read_bytes += st.scan_read_bytes
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
    achieved = alg_bytes / scan_s / 1e9 if scan_s > 0 else 0.0
    traffic, traffic_note = None, "no PMC pass for this configuration"
    if os.path.exists(PMC_TRAFFIC) and args.n_bytes == 1 << 30 and args.vocab == 32000 and world == 1:
        t = json.load(open(PMC_TRAFFIC))["traffic"]["stream_timed"]
        traffic = t["hbm_bytes_per_launch"]
        traffic_note = ("HBM bytes per timed stream-scan launch (FETCH_SIZE x2 + WRITE_SIZE, rocprofv3 PMC passes of this "
                        "command, %s): %.3g x the algorithmic bytes" % (os.path.relpath(PMC_TRAFFIC, ROOT), t["hbm_over_alg"]))
    if rank == 0:
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
                "kernel": "zbpe_scan_pairs",
                "bound": "hbm",
                "achieved": achieved,
                "peak": HBM_PEAK_GBPS,
                "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBPS,
                "traffic": traffic,
                "traffic_note": traffic_note,
                "note": "per GPU (rank 0): achieved = sum over the timed scan launches (every 8th merge, HIP events on the engine "
                        "stream) of 2 B x live tokens / sum of their durations; bytes actually streamed (block skipping, "
                        "holes) / algorithmic bytes over all launches: %.3g" % (read_bytes / max(all_alg_bytes, 1)),
            },
            "pair_count_GBps": achieved,
            "stats": {k: v for k, v in st.as_dict().items()},
            "corpus_gen_s": gen_s,
        }
        if not args.no_cpu:
            res["cpu_baseline"] = cpu_baseline(text, args.cpu_sample_bytes, args.cpu_sample_merges, args.vocab,
                                               int(st.sum_tokens), merges)
        else:
            res["cpu_baseline"] = None
        if args.scan_log_out:
            tr = eng.trace()
            with open(args.scan_log_out, "w") as f:
                json.dump({"scan_log": eng.scan_log().tolist(),
                           "live": tr[:, zbpe.TRACE_COLUMNS.index("live")].astype(np.int64).tolist()}, f)
        if args.stats_out:
            with open(args.stats_out, "w") as f:
                json.dump({"merges": m.tolist(), "counts": c.tolist()}, f)
        print(json.dumps(res), flush=True)
    eng.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
