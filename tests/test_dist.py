"""Multi-rank (sharded) training. CPU: the host-collective plumbing with gloo, world_size 2.
GPU: 2, 3, 4 and 8 ranks sharing one MI355X (collectives through gloo) must give the oracle's merges --
shard boundaries (7 of them at world 8, self-pair run parities chained across all of them), the
first-occurrence min-reduce over every rank, ties resolved by the exact path -- and C3 (world 8) and C4
(worlds 2 and 4) must equal their full goldens across the replication hand-over."""

import numpy as np
import pytest

import oracle as O
import zbpe
from dist_worker import bench_setup_worker, big_worker, collective_worker, run, train_worker


def test_host_collective_gloo_world2():
    out = run(collective_worker, 2)
    for r in (0, 1):
        _, a, m, g = out[r]
        assert a == [3, 10, (0xFFFFFFFF + 0xFFFFFFFE) & 0xFFFFFFFF]
        assert m == [5, 6, 123]
        assert g == [0, 1, 2, 200, 1, 2, 3, 200]


@pytest.mark.parametrize("case", [{}, {"share_gpu": True}, {"rccl_fails": True}], ids=["rccl", "share_gpu", "rccl_fails"])
def test_bench_multi_rank_setup_gloo_world2(case):
    """bench.py --gpus 2 engine set-up over gloo (CPU): rank 0's RCCL unique id reaches rank 1, each rank
    opens its own device with its rank; --share-gpu and an RCCL failure use host collectives."""
    out = run(bench_setup_worker, 2, case)
    for r in (0, 1):
        _, made, backend = out[r]
        assert len(made) == 1 and made[0]["rank"] == r and made[0]["world"] == 2
        if case.get("share_gpu"):
            assert backend.startswith("gloo") and made[0]["collective"] and made[0]["device"] == 0
        elif case.get("rccl_fails"):
            assert backend.startswith("gloo") and made[0]["collective"] and made[0]["device"] == r
        else:
            assert backend == "rccl" and made[0]["device"] == r
            assert made[0]["unique_id"].startswith(b"uid-of-rank-0")


CASES = [
    dict(kind="words_utf8", seed=61, n=300000, vocab=700),
    dict(kind="runs", seed=62, n=60000, vocab=400),          # (a,a) runs crossing shard boundaries
    dict(kind="uniform", seed=63, n=3000, vocab=900),         # trained to exhaustion, many ties
    dict(text=b"aaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaa", vocab=300),
    dict(text=b"abababababababababababab", vocab=300),
    dict(text=b"hello world hello", vocab=300),
    dict(text=b"ab", vocab=300),
    # occurrence lists from the first compaction: the ranks gather the stream and finish as replicas
    dict(kind="words_utf8", seed=65, n=200000, vocab=900, options={"list_start": 0}, replicated=True),
    dict(kind="runs", seed=66, n=60000, vocab=500, options={"list_start": 0}, replicated=True),
    # the same without the late-phase replication (every merge sharded to the end)
    dict(kind="words_utf8", seed=65, n=200000, vocab=900, options={"list_start": 0, "replicate_late": 0}),
    # a shrunken occurrence arena: halts and compactions are decided on replicated bounds (every rank
    # alike), and a global top count above the arena grows it on every rank (run-heavy: skewed counts)
    dict(kind="runs", seed=67, n=60000, vocab=450, options={"arena_cap": 3000, "replicate_late": 0}),
    dict(text=b"ab" * 20000 + b"xy" * 3000, vocab=320, options={"arena_cap": 12000, "replicate_late": 0}),
    # skewed shards (rank 0 words, the rest random bytes): one shard's holes pile up while another's do not;
    # compactions are decided on replicated totals, so the ranks' arena fills stay equal
    dict(parts=[("words_utf8", 68, 150000), ("uniform", 69, 150000)], vocab=700, options={"arena_cap": 40000}),
    dict(parts=[("words_utf8", 68, 150000), ("uniform", 69, 150000)], vocab=700,
         options={"arena_cap": 40000, "replicate_late": 0, "list_start": 0}),
]


def case_text(case) -> bytes:
    if "text" in case:
        return case["text"]
    if "parts" in case:
        return b"".join(zbpe.synth_corpus(k, s, n) for k, s, n in case["parts"])
    return zbpe.synth_corpus(case["kind"], case["seed"], case["n"])


def case_id(c) -> str:
    name = c.get("kind", "parts" if "parts" in c else "text") + str(c.get("n", len(c.get("text", b""))))
    return name + "".join(f"-{k}{v}" for k, v in c.get("options", {}).items())


# worlds 4 and 8 (BASELINE config 4 is chunk-sharded over 8 MI355X): the cases whose shards interact most --
# words (lists, replication), run-heavy (self-pair parities across 3 and 7 shard edges), sharded to the end,
# a shrunken arena that must grow, skewed shards, and tiny texts where most of the 8 shards are empty
WIDE = [CASES[0], CASES[1], CASES[3], CASES[6], CASES[7], CASES[9], CASES[10], CASES[13]]


@pytest.mark.gpu
@pytest.mark.parametrize("world,case", [(w, c) for w in (2, 3) for c in CASES] + [(w, c) for w in (4, 8) for c in WIDE],
                         ids=lambda x: f"w{x}" if isinstance(x, int) else case_id(x))
def test_sharded_training_matches_oracle(world, case):
    text = case_text(case)
    ref = O.train(text, case["vocab"])
    out = run(train_worker, world, case)
    for r in range(world):
        _, m, c, st = out[r][:4]
        assert m == ref.merges.tolist(), f"rank {r}"
        assert c == ref.counts.tolist(), f"rank {r}"
    assert out[0][3]["final_tokens"] == len(ref.tokens)
    # sum over merges of the stream length (the oracle also counts a final early-stop pass, n <= 1)
    assert 0 <= ref.stats.pair_tokens - out[0][3]["sum_tokens"] <= 1
    if case.get("replicated"):
        assert all(out[r][3]["replications"] == 1 for r in range(world))



@pytest.mark.gpu
@pytest.mark.parametrize("case", [CASES[0], CASES[1], CASES[9], CASES[-1]], ids=case_id)
def test_one_rank_host_collective_runs_sharded_path(case):
    """world 1 with a host collective: the sharded code path (every collective, over one rank)"""
    text = case_text(case)
    ref = O.train(text, case["vocab"])
    out = run(train_worker, 1, case)
    assert out[0][1] == ref.merges.tolist() and out[0][2] == ref.counts.tolist()
    assert out[0][3]["sharded_merges"] > 0


@pytest.mark.gpu
@pytest.mark.parametrize("options", [{}, {"replicate_late": 0, "list_start": 0}, {"exact_ties": 1}],
                         ids=["replicate_late", "sharded_to_the_end", "exact_ties"])
def test_rccl_one_rank_communicator(options):
    """A one-rank RCCL communicator (zbpe_create_dist, world 1): ncclAllReduce / ncclAllGather run on the
    engine stream every merge (count deltas, boundaries, first occurrences, stream gather), merges equal
    the oracle's; the full recount all-reduces through RCCL too"""
    text = zbpe.synth_corpus("words_utf8", 71, 300000)
    ref = O.train(text, 700)
    e = zbpe.Engine(0, rank=0, world=1, unique_id=zbpe.comm_unique_id())
    try:
        for k, v in options.items():
            e.set_option(k, v)
        m, c, st = e.train(text, 700)
        assert m.tolist() == ref.merges.tolist() and c.tolist() == ref.counts.tolist()
        assert st.sharded_merges > 0
        if not options.get("exact_ties"):  # (batched merges: the all-reduce's device time, from the timed merges)
            assert st.comm_s > 0
        if options.get("replicate_late", 1) and not options.get("exact_ties"):
            assert st.replications == 1
        assert e.verify_counts() == 0
    finally:
        e.close()


@pytest.mark.gpu
def test_sharded_exact_tie_path():
    case = dict(kind="uniform", seed=64, n=20000, vocab=600, options={"exact_ties": 1})
    text = zbpe.synth_corpus(case["kind"], case["seed"], case["n"])
    ref = O.train(text, case["vocab"])
    out = run(train_worker, 2, case)
    assert out[0][1] == ref.merges.tolist()
    assert out[0][3]["tie_fallbacks"] == out[0][3]["tie_iterations"] > 0


@pytest.mark.gpu
@pytest.mark.timeout(900)
def test_sharded_corpus_over_4GiB(tmp_path):
    """A 4.5 GiB corpus (more than 2^32 bytes) on 2 ranks: positions are shard-local u32, global order is
    (rank, local position), cross-rank sums are exact. Merge 1 must be the oracle's first iteration on the
    whole byte stream, merge 2 the oracle's iteration on the two shards' streams after merge 1."""
    case = dict(kind="words_utf8", seed=0x5EED0006, n=(9 << 29), vocab=258, dir=str(tmp_path))
    out = run(big_worker, 2, case, timeout=800)
    m, c = out[0][1], out[0][2]
    assert out[1][1] == m and out[1][2] == c and len(m) == 2
    text = zbpe.synth_corpus(case["kind"], case["seed"], case["n"], threads=8)
    r0 = O.step(np.frombuffer(text, np.uint8).astype(np.uint16))
    del text
    assert (r0.pair, r0.count) == ((m[0][0], m[0][1]), c[0])
    t = np.concatenate([np.load(tmp_path / "tok0.npy"), np.load(tmp_path / "tok1.npy")])  # after merge 1
    r1 = O.step(t)
    assert (r1.pair, r1.count) == ((m[1][0], m[1][1]), c[1])


def handover_merge(g: dict, n_bytes: int, world: int, list_start: int = 64, power: int = 2) -> int:
    """the first merge k at which the sharded ranks may replicate (Engine::run_batch, option handover = power): the top
    count times list_start times world^power is below the live tokens before merge k (the golden's counts and stream
    lengths)"""
    live = [n_bytes] + g["len_after"]
    return next(k for k in range(len(g["counts"])) if g["counts"][k] * list_start * world ** power < live[k])


def check_sharded_vs_golden(g: dict, case: dict, world: int, timeout: int):
    """`world` ranks sharing the GPU (host collectives) train the case's corpus: every rank's merges and counts
    equal the golden; the run crosses the replication hand-over, which happens at the first batch start at or
    after the golden's hand-over merge (batches hold up to 32 merges); every rank shards the same merges and
    compacts at the same merges on the same replicated arena fill. Returns the sharded merge count."""
    out = run(train_worker, world, case, timeout=timeout)
    K = g["n_merges"]
    k0 = handover_merge(g, case["n"], world)
    for r in range(world):
        _, m, c, st, clog = out[r]
        assert len(m) == case["vocab"] - 256
        assert m[:K] == g["merges"] and c[:K] == g["counts"], f"rank {r}"
        assert st["replications"] == 1 and k0 <= st["sharded_merges"] < k0 + 32, (r, st["sharded_merges"], k0)
        assert out[r][1] == out[0][1] and out[r][2] == out[0][2]
        assert st["sharded_merges"] == out[0][3]["sharded_merges"]
        assert out[r][4] == out[0][4] and len(out[r][4]) >= 2  # compactions: same merges, same replicated arena fill
    if g["complete"]:
        assert out[0][3]["final_tokens"] == g["len_after"][-1]
    print(f"HANDOVER corpus={case['n']} world={world} golden_handover={k0} sharded_merges={out[0][3]['sharded_merges']} "
          f"sharded_s={out[0][3]['sharded_s']:.3f} replicate_s={out[0][3]['replicate_s']:.3f} replicated_s={out[0][3]['replicated_s']:.3f}")
    return out[0][3]["sharded_merges"]


def _golden(name):
    import json
    import os

    from helpers import GOLDEN

    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


# the full-golden sharded runs are part of the default -m gpu suite: with the ranks sharing one GPU and host
# collectives they take seconds each (profiles/r05_pytest_dist_long.log: C4 w2 ~6 s, C4 w4 ~9 s, C3 w8 ~25 s,
# corpus generation included)


@pytest.mark.gpu
@pytest.mark.timeout(1100)
@pytest.mark.parametrize("world", [2, 4])
def test_sharded_c4_vs_golden(world):
    """C4 itself (1 GiB, vocab 32000) over 2 and 4 ranks sharing the GPU: the full C4 golden (all 31,744 merges,
    counts, final length), across the replication hand-over"""
    g = _golden("large_c4_words_utf8_1GiB_v32000.json")
    check_sharded_vs_golden(g, dict(kind="words_utf8", seed=0x5EED0004, n=1 << 30, vocab=32000), world, 1000)


@pytest.mark.gpu
@pytest.mark.timeout(600)
def test_sharded_c3_world8_vs_golden():
    """C3 (64 MiB, vocab 4096) over 8 ranks sharing the GPU: the full C3 golden (all 3,840 merges, counts, final
    length); 7 shard edges, the 8-way first-occurrence min-reduce of every exact tie in the sharded phase"""
    g = _golden("large_c3_words_utf8_64MiB_v4096.json")
    check_sharded_vs_golden(g, dict(kind="words_utf8", seed=0x5EED0003, n=64 << 20, vocab=4096), 8, 550)
