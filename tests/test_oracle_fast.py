"""CPU tests of the second oracle (oracle/zig_fast.cpp: exact incremental counts + a literal Zig-map replay
at every tied merge), which made the full C4 golden. It is pinned here against the literal oracle
(oracle/zig_ref.c, itself pinned by the reference's merges.txt and Zig's Wyhash vectors):

  - its restated Zig hash and map sizing equal zig_ref.c's;
  - on C1 (taylorswift.txt, V=300: the reference's merges.txt) and every synthetic golden it gives the literal
    oracle's merges, counts, tie counts, distinct-pair counts and final stream, both with every tie replayed
    before its merge and with the replays speculative on worker threads (restart on disagreement);
  - on C3 (64 MiB, V=4096, 1,221 ties) it reproduces the literal oracle's full-sequence golden, checkpoints
    included;
  - its C4 golden (all 31,744 merges) agrees with the literal oracle's C4 prefix in every field.
"""
import json
import os

import numpy as np
import pytest

import oracle as O
from helpers import GOLDEN, c1_text, synth_goldens, synth_text

C4_FULL = "large_c4_words_utf8_1GiB_v32000.json"
C4_PREFIX = "large_c4_words_utf8_1GiB_v32000_prefix.json"
C3_GOLDEN = "large_c3_words_utf8_64MiB_v4096.json"


def _golden(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


def test_fast_hash_and_capacity_match_zig_ref():
    L = O.fast_lib()
    k = 0x12345
    for _ in range(2000):
        assert L.zfast_pair_hash(k) == O.pair_hash(k & 0xFFFF, k >> 16)
        k = (k * 2654435761 + 12345) & 0x7FFF7FFF
    # hello world hello: D = 12 == max_load(16) and a getOrPut follows the last insertion -> capacity 32
    assert L.zfast_final_capacity(12, 1) == 32 and L.zfast_final_capacity(12, 0) == 16
    for d in (1, 6, 7, 12, 13, 25, 26, 100, 1000, 52428, 52429):
        toks = np.arange(d + 1, dtype=np.uint16)  # d distinct pairs, the last pair a first occurrence
        _, _, _, cap = O.map_order(toks)
        assert L.zfast_final_capacity(d, 0) == cap, d


def _same(r, z):
    assert np.array_equal(r.merges, z.merges)
    assert np.array_equal(r.counts, z.counts)
    assert np.array_equal(r.ties, z.ties)
    assert np.array_equal(r.distinct, z.distinct)
    assert np.array_equal(r.tokens, z.tokens)


@pytest.mark.parametrize("sync_limit", [1 << 40, 0], ids=["replay-before-merge", "speculative"])
def test_fast_oracle_equals_literal_on_c1(sync_limit):
    text = c1_text()
    r = O.fast_train(text, 300, threads=4, sync_limit=sync_limit)
    _same(r, O.train(text, 300))
    assert r.ties_sync + r.ties_async == int(np.sum(r.ties > 1)) >= 1


@pytest.mark.parametrize("g", synth_goldens(), ids=lambda g: g["name"])
@pytest.mark.parametrize("sync_limit", [1 << 40, 0], ids=["replay-before-merge", "speculative"])
def test_fast_oracle_equals_literal_on_goldens(g, sync_limit):
    text = synth_text(g)
    r = O.fast_train(text, g["vocab_size"], threads=4, sync_limit=sync_limit)
    _same(r, O.train(text, g["vocab_size"]))
    assert r.merges.astype(int).tolist() == g["merges"]
    assert r.ties_sync + r.ties_async == int(np.sum(r.ties > 1))


def test_fast_oracle_edge_inputs():
    for text, vocab in ((b"", 300), (b"a", 300), (b"aaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaa", 300), (bytes(range(256)) * 3, 400),
                        (b"abababababababab" * 7, 280)):
        _same(O.fast_train(text, vocab, threads=2, sync_limit=0), O.train(text, vocab))
    with pytest.raises(ValueError):
        O.fast_train(b"abc", 255)


def test_fast_oracle_reproduces_c3_golden(tmp_path):
    """all 3,840 C3 merges with their counts, ties, distinct pairs and lengths, and every FNV checkpoint"""
    import zbpe

    g = _golden(C3_GOLDEN)
    text = zbpe.synth_corpus(g["kind"], g["seed"], g["n"], threads=8)
    log = tmp_path / "c3.log"
    r = O.fast_train(text, g["vocab_size"], threads=8, fnv_every=64, progress=str(log))
    assert r.merges.astype(int).tolist() == g["merges"]
    assert r.counts.astype(int).tolist() == g["counts"]
    assert r.ties.astype(int).tolist() == g["ties"]
    assert r.distinct.astype(int).tolist() == g["distinct"]
    assert r.len_after.astype(int).tolist() == g["len_after"]
    fnv = {int(p[1]): p[3] for p in (line.split() for line in open(log)) if p and p[0] in ("fnv", "done")}
    assert all(fnv[k] == h for k, _, h in g["fnv64_after"])
    assert r.restarts == 0 and r.ties_sync + r.ties_async == sum(t > 1 for t in g["ties"]) == 1221


def test_c4_full_golden_agrees_with_literal_prefix():
    """the fast oracle's full C4 run (31,744 merges) and the literal oracle's prefix agree on every field of
    every merge the prefix holds and on every shared FNV checkpoint; invariants of the whole run"""
    if not os.path.exists(os.path.join(GOLDEN, C4_FULL)):
        pytest.skip("full C4 golden not generated yet (tests/golden/make_golden_large.py run-fast c4)")
    full, pre = _golden(C4_FULL), _golden(C4_PREFIX)
    assert full["complete"] and full["n_merges"] == 32000 - 256 and full["corpus_sha256"] == pre["corpus_sha256"]
    K = pre["n_merges"]
    assert K >= 1000
    for f in ("merges", "counts", "ties", "distinct", "len_after"):
        assert full[f][:K] == pre[f], f
    fp = {k: (ln, h) for k, ln, h in full["fnv64_after"]}
    shared = [(k, ln, h) for k, ln, h in pre["fnv64_after"] if k in fp]
    assert len(shared) >= 10 and all(fp[k] == (ln, h) for k, ln, h in shared)
    m, c, ln = full["merges"], full["counts"], full["len_after"]
    assert [x for _, _, x in m] == list(range(256, 32000))
    assert all(c[i] >= c[i + 1] for i in range(len(c) - 1))
    prev = full["n"]
    for (a, b, _), cnt, after in zip(m, c, ln):
        assert after == prev - cnt if a != b else prev - cnt <= after < prev
        prev = after
    # every tie was confirmed by a literal map replay, none overruled the run
    assert full["tie_replays"]["mismatches"] == 0 and full["tie_replays"]["restarts"] == 0
    assert full["tie_replays"]["replayed"] == sum(t > 1 for t in full["ties"])
