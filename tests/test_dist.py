"""Multi-rank (sharded) training. CPU: the host-collective plumbing with gloo, world_size 2.
GPU: 2-3 ranks sharing one MI355X (collectives through gloo) must give the oracle's merges --
shard boundaries, self-pair runs crossing shards, ties resolved by the exact path."""
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


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("case", CASES, ids=case_id)
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


@pytest.mark.gpu
@pytest.mark.timeout(1100)
def test_sharded_c4_world2_vs_golden():
    """C4 itself (1 GiB, vocab 32000) sharded over 2 ranks that share the GPU (host collectives): every merge and
    count equals the C4 golden (the fast oracle's full run when committed, else the literal oracle's prefix);
    the run crosses the replication hand-over (sharded merges, then one gather, then replicas), and both ranks
    compact at the same merges on the same replicated arena fill."""
    import json
    import os

    from helpers import GOLDEN

    full = os.path.join(GOLDEN, "large_c4_words_utf8_1GiB_v32000.json")
    path = full if os.path.exists(full) else os.path.join(GOLDEN, "large_c4_words_utf8_1GiB_v32000_prefix.json")
    with open(path) as f:
        g = json.load(f)
    case = dict(kind="words_utf8", seed=0x5EED0004, n=1 << 30, vocab=32000)
    out = run(train_worker, 2, case, timeout=1000)
    K = g["n_merges"]
    for r in (0, 1):
        _, m, c, st, clog = out[r]
        assert len(m) == 32000 - 256
        assert m[:K] == g["merges"] and c[:K] == g["counts"], f"rank {r}"
        assert st["replications"] == 1 and 0 < st["sharded_merges"] < len(m), f"rank {r}"
    assert out[0][1] == out[1][1] and out[0][2] == out[1][2]
    assert out[0][3]["sharded_merges"] == out[1][3]["sharded_merges"]
    assert out[0][4] == out[1][4] and len(out[0][4]) >= 2  # compactions: same merges, same replicated arena fill
    assert out[0][3]["final_tokens"] == g["len_after"][-1] if g["complete"] else True
