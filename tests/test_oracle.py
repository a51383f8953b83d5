"""CPU tests of the oracle (oracle/zig_ref.c) against the reference's own artefacts:
Zig wyhash.zig known-answer vectors, merges.txt (config 1), the five inline tests of
basic_tokenizer.zig:351-461 restated, and the committed seeded goldens."""
import os
import subprocess

import numpy as np
import pytest

import oracle as O
from helpers import c1_golden, c1_merges_txt, c1_text, sha256, synth_goldens, synth_text


def test_wyhash_known_answers():
    assert O.selftest() == 0  # Zig 0.13 lib/std/hash/wyhash.zig test vectors
    assert O.wyhash(0, b"") == 0x0409638EE2BDE459
    assert O.wyhash(3, b"message digest") == 0x8619124089A3A16B


@pytest.mark.parametrize("pair,h", [((0, 0), 0x14B83016DC460955), ((104, 101), 0xA96A3086990FD3BF),
                                    ((101, 32), 0x544D3DA525A0DEDA), ((46, 10), 0xDA1944F769904CC9),
                                    ((265, 101), 0x3A6CB6F333C4024E), ((256, 257), 0x61071EF1FA2190F0),
                                    ((65535, 65535), 0x53AC8FA6824BCAD0)])
def test_pair_hash(pair, h):
    assert O.pair_hash(*pair) == h


def test_c1_merges_txt_reproduced():
    g = c1_golden()
    text = c1_text()
    assert sha256(text) == g["taylorswift_sha256"]
    assert sha256(c1_merges_txt()) == g["merges_txt_sha256"] == \
        "f1a9b78b2be24bf3c6813cb0efd4920f0e40347ac7da7a098df61bd215d5f8d0"
    r = O.train(text, 300)
    assert O.serialize(r.merges) == c1_merges_txt()
    # merge 294 (line 39) is a real top-count tie decided by the Zig hash-map order
    assert r.ties[38] == 2 and r.counts[38] == 685 and list(r.merges[38]) == [265, 101, 294]


def test_hello_world_hello_map_order():
    toks = list(b"hello world hello")
    keys, slots, counts, cap = O.map_order(toks)
    assert cap == 32  # D = 12 == max_load(16) and a getOrPut follows the 12th insertion
    order = [bytes([k & 0xFF, k >> 16]) for k in keys]
    assert order == [b"wo", b"d ", b" h", b"el", b"lo", b"ld", b"o ", b" w", b"ll", b"or", b"rl", b"he"]
    r = O.train(b"hello world hello", 300)
    assert r.merges.tolist() == [[101, 108, 256], [104, 256, 257], [257, 108, 258], [258, 111, 259], [119, 111, 260],
                                 [32, 260, 261], [261, 114, 262], [100, 32, 263], [259, 262, 264], [264, 108, 265],
                                 [265, 263, 266], [266, 259, 267]]


# --- basic_tokenizer.zig:351-461 restated -------------------------------------------------------
HW_MERGES = np.array([[ord("h"), ord("e"), 256], [256, ord("l"), 257], [ord("w"), ord("o"), 258]], dtype=np.uint16)


def test_ref_generateInitialTokens():
    r = O.train(b"hello world", 256)
    assert r.tokens.tolist() == list(b"hello world")


def test_ref_encode():
    for literal in (True, False):
        assert O.encode(HW_MERGES, b"hello world", literal).tolist() == [257, ord("l"), ord("o"), ord(" "), 258, ord("r"),
                                                                         ord("l"), ord("d")]


def test_ref_decode():
    assert O.decode(HW_MERGES, [257, ord("l"), ord("o"), ord(" "), 258, ord("r"), ord("l"), ord("d")]) == b"hello world"


def test_ref_train():
    r = O.train(b"hello world hello", 300)
    assert len(r.merges) > 0
    enc = O.encode(r.merges, b"hello")
    assert enc.tolist() == [259]
    assert O.decode(r.merges, enc) == b"hello"


def test_ref_serialize_roundtrip(tmp_path):
    import zbpe

    t = zbpe.BasicTokenizer()
    for a, b, c in HW_MERGES:
        t.merges.put(zbpe.CharPair(int(a), int(b)), int(c))
    p = tmp_path / "test_merges.txt"
    t.serializeMerges(str(p))
    assert p.read_bytes() == O.serialize(HW_MERGES)
    t2 = zbpe.BasicTokenizer()
    t2.deserializeMerges(str(p))
    assert t2.merges.merges == t.merges.merges


def test_edge_cases():
    with pytest.raises(ValueError):
        O.train(b"abc", 255)
    for text in (b"", b"a"):
        assert len(O.train(text, 300).merges) == 0
    r = O.train(b"ab", 300)
    assert r.merges.tolist() == [[97, 98, 256]]
    r = O.train(b"aaaa", 300)  # self pairs: overlapping count 3, left-greedy merge -> 256 256
    assert r.counts[0] == 3 and r.merges[1].tolist() == [256, 256, 257]


def test_encode_literal_equals_linear():
    rng = np.random.default_rng(1)
    text = bytes(rng.integers(97, 100, 3000, dtype=np.uint8))
    r = O.train(text, 400)
    assert np.array_equal(O.encode(r.merges, text, True), O.encode(r.merges, text, False))
    assert np.array_equal(O.encode(r.merges, text), r.tokens)


@pytest.mark.parametrize("g", synth_goldens(), ids=lambda g: g["name"])
def test_synth_goldens(g):
    text = synth_text(g)
    r = O.train(text, g["vocab_size"])
    assert r.merges.tolist() == g["merges"]
    assert r.counts.tolist() == g["counts"]
    assert sha256(r.tokens.tobytes()) == g["final_tokens_sha256"]


def test_incremental_model_matches_oracle(tmp_path):
    """The CPU design model of the engine's incremental algorithm (tests/model/inc_model.cpp)."""
    src = os.path.join(os.path.dirname(__file__), "model", "inc_model.cpp")
    exe = tmp_path / "inc_model"
    subprocess.run(["g++", "-O2", "-std=c++17", "-o", str(exe), src], check=True)
    for g in synth_goldens():
        if g["n"] > (1 << 18):
            continue
        p = tmp_path / "c.bin"
        p.write_bytes(synth_text(g))
        out = subprocess.run([str(exe), str(p), str(g["vocab_size"])], capture_output=True, check=True).stdout
        assert out == O.serialize(np.array(g["merges"], dtype=np.uint16)), g["name"]


@pytest.mark.parametrize("literal", [False, True])
def test_step_matches_train(literal):
    """oracle.step (one expandVocabulary iteration on a given stream, used by the C3/C4 GPU parity
    tests) agrees with the full train: on the stream after k merges it picks merge k + 1, ties
    included (C1 line 39 is a tie decided by the Zig slot order)."""
    text = c1_text()
    full = O.train(text, 300)
    for k in (0, 1, 20, 38, 43):
        r = O.train(text, 256 + k)
        s = O.step(r.tokens, literal=literal)
        a, b, _ = full.merges[k]
        assert s.pair == (int(a), int(b)) and s.count == int(full.counts[k]) and s.ties == int(full.ties[k])
        assert s.distinct == int(full.distinct[k])
    for g in synth_goldens()[:3]:
        t = synth_text(g)
        r = O.train(t, 256 + 5)
        s = O.step(r.tokens, literal=literal)
        assert s.pair == tuple(g["merges"][5][:2]) and s.count == g["counts"][5]
    assert O.step(np.zeros(1, np.uint16)) is None and O.step(np.zeros(0, np.uint16)) is None


def _apply_merges_with_holes(text: bytes, merges, on_merge):
    """replaceTopPairWithNewToken (basic_tokenizer.zig:207-232) on a position-stable stream: merged-away
    slots become holes instead of being squeezed out, as in the device stream. on_merge(k, toks, alive,
    occ) sees each merge's occurrence starts before they are applied."""
    toks = np.frombuffer(text, np.uint8).astype(np.int64)
    alive = np.ones(len(toks), bool)
    for k, (a, b, x) in enumerate(np.asarray(merges, dtype=np.int64)):
        idx = np.flatnonzero(alive)
        seq = toks[idx]
        if a != b:
            occ = idx[:-1][(seq[:-1] == a) & (seq[1:] == b)]
        else:  # left-greedy over runs of a
            occ, i = [], 0
            while i + 1 < len(seq):
                if seq[i] == a and seq[i + 1] == a:
                    occ.append(idx[i])
                    i += 2
                else:
                    i += 1
            occ = np.asarray(occ, dtype=np.int64)
        on_merge(k, toks, alive, occ)
        nxt = {p: q for p, q in zip(idx[:-1], idx[1:])}
        for p in occ:
            toks[p] = x
            alive[nxt[p]] = False


@pytest.mark.parametrize("corpus", ["c1", "words_utf8"])
def test_list_neighbour_filter_invariant(corpus):
    """The filtered list walk (kernels.hpp scan_dispatch): after a list build at merge T, a position's
    successor / predecessor only ever changes into a token created after T. So for a later merge (a, b)
    with a, b both older than T, every occurrence start p had successor b at T, and its b had predecessor a."""
    import zbpe
    text = c1_text() if corpus == "c1" else zbpe.synth_corpus("words_utf8", 91, 120000)
    merges = O.train(text, 300 if corpus == "c1" else 420).merges
    builds = (5, 20)
    snap = {}
    checked = [0]

    def on_merge(k, toks, alive, occ):
        if k in builds:  # "build": each live position's live neighbours now
            idx = np.flatnonzero(alive)
            succ = np.full(len(toks), -1)
            pred = np.full(len(toks), -1)
            succ[idx[:-1]] = toks[idx[1:]]
            pred[idx[1:]] = toks[idx[:-1]]
            snap[k] = (succ, pred, 256 + k)
        a, b, _ = merges[k]
        nxt = np.flatnonzero(alive)
        pos = {int(p): i for i, p in enumerate(nxt)}
        for t, (succ, pred, lx) in snap.items():
            if a < lx and b < lx and a != b:
                assert np.all(succ[occ] == b), (k, t)
                q = nxt[[pos[int(p)] + 1 for p in occ]]
                assert np.all(pred[q] == a), (k, t)
                checked[0] += len(occ)

    _apply_merges_with_holes(text, merges, on_merge)
    assert checked[0] > 1000


def test_large_goldens_are_the_oracles_runs():
    """tests/golden/large_*.json (full-sequence C3 and the C4 prefix, made by make_golden_large.py) are
    the oracle's literal runs: their first merges recomputed here, and their internal invariants."""
    import json
    import os

    import zbpe
    from helpers import GOLDEN

    for name, first in (("large_c3_words_utf8_64MiB_v4096.json", 6), ("large_c4_words_utf8_1GiB_v32000_prefix.json", 0)):
        with open(os.path.join(GOLDEN, name)) as f:
            g = json.load(f)
        m, c, ln = g["merges"], g["counts"], g["len_after"]
        assert len(m) == len(c) == len(ln) == len(g["ties"]) == g["n_merges"] > 0
        assert [x for _, _, x in m] == list(range(256, 256 + len(m)))
        assert all(c[i] >= c[i + 1] for i in range(len(c) - 1))
        prev = g["n"]
        for (a, b, _), cnt, after in zip(m, c, ln):  # a merge removes one token per occurrence
            assert after == prev - cnt if a != b else prev - cnt <= after < prev  # (a, a): overlapping counts
            prev = after
        if first:
            text = zbpe.synth_corpus(g["kind"], g["seed"], g["n"])
            r = O.train(text, 256 + first)
            assert r.merges.astype(int).tolist() == m[:first] and r.counts.astype(int).tolist() == c[:first]
