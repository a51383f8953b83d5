"""Parity at the BASELINE.json sizes (C3, C4, C5) on the MI355X.

Unconditional, full-sequence goldens (tests/golden/large_*.json, made by make_golden_large.py: the
literal oracle run from the raw bytes in the build container):
  - C3 (64 MiB, V=4096): all 3,840 merges, their counts and the final stream's FNV-64;
  - C4 (1 GiB, V=32000): the first K merges (the oracle's prefix, ~3-9 s per literal iteration on the
    1 GiB stream), and the stream's FNV-64 after a checkpoint merge.
Exact tie cross-checks: every C3 tie, and a window of >= 50 consecutive late C4 merges, decided by
both the device's cluster test and the exact Zig-map emulation (options exact_ties /
exact_ties_from / exact_ties_to); a disagreement fails the train.

Conditional samples at any merge of C4: train to 256 + k merges, download the device's token
stream (zbpe_tokens) and ask the oracle what expandVocabulary would merge next on it (oracle.step =
basic_tokenizer.zig:183-204 once: count in the Zig map, slot order, stable sort, [0]). That must be
the full run's merge k + 1 with its count.

Size-independent properties at full size: the incremental counts equal a full recount of the final
stream (zbpe_verify_counts), encode(corpus) reproduces the training stream, decode(encode(x)) == x.
C5: encode with all 31,744 C4 merges against the oracle's encode on a 1 MiB slice of the C5 text.
"""
import hashlib
import json
import os

import numpy as np
import pytest

import oracle as O
import zbpe
from helpers import GOLDEN

pytestmark = pytest.mark.gpu

C3_SEED, C4_SEED, C5_SEED = 0x5EED0003, 0x5EED0004, 0x5EED0005


class Run:
    def __init__(self, n_bytes, seed, vocab):
        self.text = zbpe.synth_corpus("words_utf8", seed, n_bytes, threads=16)
        self.vocab = vocab
        self.e = zbpe.Engine(0)
        self.e.upload(self.text)
        self.merges, self.counts, self.stats = self.e.train_resident(vocab)
        self.log = self.e.merge_log()  # (pair, count, live tokens, tied pairs, ...) per merge
        self.mismatches = self.e.verify_counts()
        fin = self.e.tokens()
        self.final_len = len(fin)
        self.final_sha = hashlib.sha256(fin.tobytes()).hexdigest()
        self.final_fnv = O.fnv64(fin)
        self.text_sha = hashlib.sha256(self.text).hexdigest()
        del fin

    def check_step(self, k):
        """train to 256 + k; the oracle's next merge on the device stream == the full run's merge k + 1"""
        m, c, st = self.e.train_resident(256 + k)
        assert len(m) == k
        assert np.array_equal(m, self.merges[:k]) and np.array_equal(c, self.counts[:k])
        tok = self.e.tokens()
        assert len(tok) == st.final_tokens
        r = O.step(tok)
        assert r is not None
        a, b, x = (int(v) for v in self.merges[k])
        assert (r.pair, r.count) == ((a, b), int(self.counts[k])), (k, r.pair, r.count, r.ties, (a, b), self.counts[k])
        assert x == 256 + k
        return r

    def close(self):
        self.e.close()


def large_golden(name: str) -> dict:
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


def check_vs_golden(run: Run, g: dict, k: int):
    """the run's first k merges and counts == the oracle's (unconditional: both from the raw bytes)"""
    assert run.text_sha == g["corpus_sha256"], "corpus generator changed"
    assert run.merges[:k].astype(int).tolist() == g["merges"][:k]
    assert run.counts[:k].astype(int).tolist() == g["counts"][:k]


def decode_np(merges: np.ndarray, tokens: np.ndarray) -> bytes:
    """decode (basic_tokenizer.zig:90-138) vectorised: the byte expansion of every token id (first
    merge with that new_token wins, like findMerge), gathered for the whole stream."""
    first = {}
    for i, (a, b, x) in enumerate(merges.tolist()):
        first.setdefault(x, (a, b))
    exp = {t: bytes([t]) for t in range(256)}
    for x in sorted(first):
        a, b = first[x]
        exp[x] = exp[a] + exp[b]
    vmax = max(exp) + 1
    lens = np.zeros(vmax, np.int64)
    offs = np.zeros(vmax, np.int64)
    flat = bytearray()
    for t in range(vmax):
        if t in exp:
            offs[t] = len(flat)
            lens[t] = len(exp[t])
            flat += exp[t]
    flat = np.frombuffer(bytes(flat), np.uint8)
    tk = tokens.astype(np.int64)
    ln = lens[tk]
    assert np.all(ln > 0), "token without a merge (InvalidToken)"
    starts = np.cumsum(ln) - ln
    idx = np.repeat(offs[tk] - starts, ln) + np.arange(int(ln.sum()))
    return flat[idx].tobytes()


@pytest.fixture(scope="module")
def c4():
    r = Run(1 << 30, C4_SEED, 32000)
    yield r
    r.close()


@pytest.fixture(scope="module")
def c3():
    r = Run(64 << 20, C3_SEED, 4096)
    yield r
    r.close()


# --- C4: 1 GiB, vocab 32000 (the bench workload) -----------------------------------------------------
def test_c4_full_run_properties(c4):
    assert len(c4.merges) == 32000 - 256
    assert c4.merges[:, 2].tolist() == list(range(256, 32000))
    assert np.all(np.diff(c4.counts.astype(np.int64)) <= 0)  # the top count never increases
    assert c4.mismatches == 0  # incremental counts == full recount of the final stream
    assert c4.stats.final_tokens == c4.final_len


C4_GOLDEN = "large_c4_words_utf8_1GiB_v32000_prefix.json"
C3_GOLDEN = "large_c3_words_utf8_64MiB_v4096.json"


def test_c4_prefix_vs_oracle_golden(c4):
    """the first K merges of C4 (the oracle's literal run from the 1 GiB of bytes) bit-exact, ties
    included, and the device stream after the last checkpoint equal to the oracle's (FNV-64)"""
    g = large_golden(C4_GOLDEN)
    K = g["n_merges"]
    assert K >= 500
    check_vs_golden(c4, g, K)
    k, ln, fnv = [x for x in g["fnv64_after"] if x[0] <= K][-1]
    m, c, st = c4.e.train_resident(256 + k)
    tok = c4.e.tokens()
    assert len(tok) == ln and O.fnv64(tok) == int(fnv, 16)


C4_FULL = "large_c4_words_utf8_1GiB_v32000.json"


def test_c4_full_sequence_vs_oracle_golden(c4):
    """all 31,744 C4 merges and counts equal the full golden (oracle/zig_fast.cpp: exact incremental counts, every
    one of the ~20,000 tied merges decided by a literal Zig-map replay; it agrees with the literal oracle's
    prefix, tests/test_oracle_fast.py), with the same tied merges; the final stream's length and FNV-64, and the
    device stream at checkpoints spread over the run"""
    if not os.path.exists(os.path.join(GOLDEN, C4_FULL)):
        pytest.skip("full C4 golden not committed")
    g = large_golden(C4_FULL)
    assert g["complete"] and g["n_merges"] == 31744 and g["tie_replays"]["mismatches"] == 0
    check_vs_golden(c4, g, 31744)
    assert c4.stats.tie_iterations == sum(t > 1 for t in g["ties"])
    assert c4.log[:, 3].astype(int).tolist() == g["ties"]  # every merge's tied-pair count (rounds derive them)
    assert c4.log[:, 1].astype(int).tolist() == g["counts"]
    # the multi-merge rounds ran (a gate change that switched them off would otherwise leave this green):
    # round 5 measured ~15,000 merges applied beyond the rounds' first members
    assert c4.stats.round_merges > 10000, c4.stats.round_merges
    k, ln, fnv = g["fnv64_after"][-1]
    assert k == 31744 and c4.final_len == ln and c4.final_fnv == int(fnv, 16)
    cps = {k: (ln, h) for k, ln, h in g["fnv64_after"]}
    for k in (2048, 8192, 16384, 24576, 30720):
        ln, h = cps[k]
        _, _, st = c4.e.train_resident(256 + k)
        tok = c4.e.tokens()
        assert len(tok) == ln and O.fnv64(tok) == int(h, 16), k


def test_c4_late_ties_exact_window(c4):
    """SELF-CONSISTENCY CHECK, not oracle evidence (the full C4 golden above is): >= 50 consecutive late C4
    tie decisions (merges 25,000-25,069) taken by both the device's cluster test and the product's own exact
    Zig-map emulation (first occurrences of all ~4e7 live pairs); a disagreement fails the train; the merges
    equal the production run's"""
    e = c4.e
    e.set_option("exact_ties_from", 25000)
    e.set_option("exact_ties_to", 25070)
    try:
        m, c, st = e.train_resident(32000)
    finally:
        e.set_option("exact_ties_to", 0)
    assert np.array_equal(m, c4.merges) and np.array_equal(c, c4.counts)
    assert st.tie_crosschecks == st.tie_fallbacks >= 50


@pytest.mark.parametrize("k", [0, 1, 2, 100, 1000, 1400, 2500, 5000, 10000, 15000, 20000, 25000, 31000, 31743])
def test_c4_oracle_step(c4, k):
    c4.check_step(k)


def test_c4_encode_equals_training_stream(c4):
    enc = c4.e.encode(c4.merges, c4.text)
    assert len(enc) == c4.final_len
    assert hashlib.sha256(enc.tobytes()).hexdigest() == c4.final_sha


def test_c5_encode_slice_vs_oracle(c4):
    """C5 (encode 100 M chars with the 31,744 C4 merges): a 1 MiB slice against the oracle's encode."""
    text = zbpe.synth_corpus("words_utf8", C5_SEED, 100_000_000, threads=16)
    piece = text[37_000_000:37_000_000 + (1 << 20)]
    assert np.array_equal(c4.e.encode(c4.merges, piece), O.encode(c4.merges, piece))


def test_c5_encode_full_round_trip(c4):
    """C5 at full size: decode(encode(text)) == text, and the encoding is shorter than the text."""
    text = zbpe.synth_corpus("words_utf8", C5_SEED, 100_000_000, threads=16)
    enc = c4.e.encode(c4.merges, text)
    assert 0 < len(enc) < len(text) // 2
    assert decode_np(c4.merges, enc) == text


# --- C3: 64 MiB, vocab 4096 -----------------------------------------------------------------------
def test_c3_full_run_properties(c3):
    assert len(c3.merges) == 4096 - 256
    assert c3.merges[:, 2].tolist() == list(range(256, 4096))
    assert all(int(a) < int(x) and int(b) < int(x) for a, b, x in c3.merges)
    assert np.all(np.diff(c3.counts.astype(np.int64)) <= 0)
    assert c3.mismatches == 0
    # the first merge against the oracle's count of the whole 64 MiB byte stream
    r = O.step(np.frombuffer(c3.text, np.uint8).astype(np.uint16))
    assert (r.pair, r.count) == ((int(c3.merges[0, 0]), int(c3.merges[0, 1])), int(c3.counts[0]))


def test_c3_full_sequence_vs_oracle_golden(c3):
    """all 3,840 C3 merges and counts equal the oracle's literal run from the 64 MiB of bytes, and the
    final stream equals the oracle's (FNV-64 and length)"""
    g = large_golden(C3_GOLDEN)
    assert g["complete"] and g["n_merges"] == 3840
    check_vs_golden(c3, g, 3840)
    assert c3.log[:, 3].astype(int).tolist() == g["ties"]
    k, ln, fnv = g["fnv64_after"][-1]
    assert k == 3840 and c3.final_len == ln and c3.final_fnv == int(fnv, 16)
    assert c3.stats.round_merges > 0, "multi-merge rounds did not run on C3"


def test_c3_every_tie_exact(c3):
    """every C3 tie (1,221) decided by both the cluster test and the exact Zig-map emulation"""
    g = large_golden(C3_GOLDEN)
    e = c3.e
    e.set_option("exact_ties", 1)
    try:
        m, c, st = e.train_resident(4096)
    finally:
        e.set_option("exact_ties", 0)
    assert np.array_equal(m, c3.merges) and np.array_equal(c, c3.counts)
    tied = sum(t > 1 for t in g["ties"])
    assert st.tie_iterations == st.tie_fallbacks == st.tie_crosschecks == tied > 1000


@pytest.mark.parametrize("k", [1, 37, 500, 2000, 3839])
def test_c3_oracle_step(c3, k):
    c3.check_step(k)


def test_c3_encode_and_decode(c3):
    enc = c3.e.encode(c3.merges, c3.text)
    assert len(enc) == c3.final_len
    assert hashlib.sha256(enc.tobytes()).hexdigest() == c3.final_sha
    assert decode_np(c3.merges, enc) == c3.text
    t = zbpe.BasicTokenizer()
    for a, b, x in c3.merges:
        t.merges.put(zbpe.CharPair(int(a), int(b)), int(x))
    pre = c3.text[: 1 << 18]
    assert t.decode(c3.e.encode(c3.merges, pre)) == pre  # the API's own decode on a prefix


# --- pair selects and chains: fewer launches' work, the same merges -------
PAIR_OPTS = [
    {"pair_select": 0},
    {"pair_select": 1, "pair_chain": 0},
    {"pair_select": 1, "pair_chain": 1},
    {"pair_select": 1, "pair_chain": 2},
    {"pair_select": 1, "pair_chain": 3},
    {"pair_select": 1, "pair_refresh": 1},
]


def _train_with(text, vocab, opts):
    e = zbpe.Engine(0)
    e.upload(text)
    try:
        for k, v in opts.items():
            e.set_option(k, v)
    except Exception:
        e.close()
        raise
    m, c, st = e.train_resident(vocab)
    fnv = O.fnv64(e.tokens())
    mism = e.verify_counts()
    e.close()
    return m, c, st, fnv, mism


@pytest.mark.parametrize("opts", PAIR_OPTS, ids=lambda o: ",".join(f"{k}={v}" for k, v in o.items()))
def test_c3_pair_options_same_run(c3, opts):
    """every C3 merge, count and tie count, the final stream and the recount are the same whichever of the
    pair options is on; the counters say the option did something"""
    m, c, st, fnv, mism = _train_with(c3.text, c3.vocab, opts)
    assert np.array_equal(m, c3.merges) and np.array_equal(c, c3.counts)
    assert st.tie_iterations == c3.stats.tie_iterations
    assert fnv == c3.final_fnv and mism == 0
    if opts.get("pair_select", 1):
        assert st.pair_selects > 0
    else:
        assert st.pair_selects == 0


def test_c4_pair_chain_depths_same_run(c4):
    """C4 with chains of depth 1 and 3 (the default is 2), untied rounds off so that the batches outside tied
    streaks take pair selects: all 31,744 merges and counts, the tie count, the final stream; the deeper chain
    takes more pair selects"""
    sel = {}
    for depth in (1, 3):
        m, c, st, fnv, mism = _train_with(c4.text, c4.vocab, {"pair_chain": depth, "round_untied": 0})
        assert np.array_equal(m, c4.merges) and np.array_equal(c, c4.counts)
        assert st.tie_iterations == c4.stats.tie_iterations
        assert fnv == c4.final_fnv and mism == 0
        sel[depth] = st.pair_selects
    assert sel[3] > sel[1] > 0, sel


# --- multi-merge rounds: the same run whatever the round size -------------------
ROUND_OPTS = [
    {"round_k": 1},
    {"round_k": 2, "round_ties": 0},
    {"round_k": 5, "round_ties": 0},
    {"round_k": 5, "round_ties": 0, "pair_chain": 0},
    {"round_k": 5, "round_untied": 0},  # tied rounds only (the round-5 form)
    {"round_k": 3, "round_ties": 100},  # untied rounds, tied ones only in all-tied batches
]


@pytest.mark.parametrize("opts", ROUND_OPTS, ids=lambda o: ",".join(f"{k}={v}" for k, v in o.items()))
def test_c3_round_sizes_same_run(c3, opts):
    """C3 with rounds off (round_k 1), rounds of two, and rounds of five in every list streak (round_ties 0, with
    and without pair chains): every merge, count and per-merge tie count of the golden, the final stream (FNV-64)
    and a full recount; the rounds ran exactly when enabled"""
    g = large_golden(C3_GOLDEN)
    e = zbpe.Engine(0)
    e.upload(c3.text)
    try:
        for k, v in opts.items():
            e.set_option(k, v)
        m, c, st = e.train_resident(c3.vocab)
        log = e.merge_log()
        fnv = O.fnv64(e.tokens())
        mism = e.verify_counts()
    finally:
        e.close()
    assert m.astype(int).tolist() == g["merges"] and c.astype(int).tolist() == g["counts"]
    assert log[:, 3].astype(int).tolist() == g["ties"]
    assert fnv == c3.final_fnv and mism == 0
    assert (st.round_merges > 0) == (opts["round_k"] > 1), st.round_merges


@pytest.mark.parametrize("untied", [0, 1])
def test_c4_untied_rounds_same_run(c4, untied):
    """C4 with untied rounds off and on: all 31,744 merges, counts and per-merge tie counts, the final stream and the
    recount are the fixture's; with them on, untied rounds merged members (the mid phase's merges are mostly untied)"""
    e = zbpe.Engine(0)
    e.upload(c4.text)
    try:
        e.set_option("round_untied", untied)
        m, c, st = e.train_resident(c4.vocab)
        log = e.merge_log()
        fnv = O.fnv64(e.tokens())
        mism = e.verify_counts()
    finally:
        e.close()
    assert np.array_equal(m, c4.merges) and np.array_equal(c, c4.counts)
    assert np.array_equal(log[:, 3], c4.log[:, 3])
    assert fnv == c4.final_fnv and mism == 0
    assert st.round_merges > 0

