"""Multi-rank (sharded) training. CPU: the host-collective plumbing with gloo, world_size 2.
GPU: 2-3 ranks sharing one MI355X (collectives through gloo) must give the oracle's merges --
shard boundaries, self-pair runs crossing shards, ties resolved by the exact path."""
import numpy as np
import pytest

import oracle as O
import zbpe
from dist_worker import collective_worker, run, train_worker


def test_host_collective_gloo_world2():
    out = run(collective_worker, 2)
    for r in (0, 1):
        _, a, m, g = out[r]
        assert a == [3, 10, (0xFFFFFFFF + 0xFFFFFFFE) & 0xFFFFFFFF]
        assert m == [5, 6, 123]
        assert g == [0, 1, 2, 200, 1, 2, 3, 200]


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
]


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("case", CASES, ids=lambda c: c.get("kind", "text") + str(c.get("n", len(c.get("text", b""))))
                         + "".join(f"-{k}{v}" for k, v in c.get("options", {}).items()))
def test_sharded_training_matches_oracle(world, case):
    text = case["text"] if "text" in case else zbpe.synth_corpus(case["kind"], case["seed"], case["n"])
    ref = O.train(text, case["vocab"])
    out = run(train_worker, world, case)
    for r in range(world):
        _, m, c, st = out[r]
        assert m == ref.merges.tolist(), f"rank {r}"
        assert c == ref.counts.tolist(), f"rank {r}"
    assert out[0][3]["final_tokens"] == len(ref.tokens)
    # sum over merges of the stream length (the oracle also counts a final early-stop pass, n <= 1)
    assert 0 <= ref.stats.pair_tokens - out[0][3]["sum_tokens"] <= 1
    if case.get("replicated"):
        assert all(out[r][3]["replications"] == 1 for r in range(world))



@pytest.mark.gpu
def test_sharded_exact_tie_path():
    case = dict(kind="uniform", seed=64, n=20000, vocab=600, options={"exact_ties": 1})
    text = zbpe.synth_corpus(case["kind"], case["seed"], case["n"])
    ref = O.train(text, case["vocab"])
    out = run(train_worker, 2, case)
    assert out[0][1] == ref.merges.tolist()
    assert out[0][3]["tie_fallbacks"] == out[0][3]["tie_iterations"] > 0
