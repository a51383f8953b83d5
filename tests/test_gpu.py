"""Parity tests on the MI355X: the HIP path (libzbpe.so through the C ABI) against the oracle's
merges on the same inputs -- bit-exact merges and per-merge counts, at sizes the oracle finishes
in seconds, plus size-independent properties at larger sizes."""
import numpy as np
import pytest

import oracle as O
import zbpe
from helpers import c1_golden, c1_merges_txt, c1_text, synth_goldens, synth_text

pytestmark = pytest.mark.gpu


def _train(engine, text, vocab):
    m, c, st = engine.train(text, vocab)
    return m, c, st


def test_c1_taylorswift_bit_exact(engine):
    g = c1_golden()
    m, c, st = _train(engine, c1_text(), 300)
    assert zbpe.merges_to_text(m) == c1_merges_txt()
    assert c.tolist() == g["oracle_counts"]
    assert st.final_tokens == g["oracle_final_tokens"]
    assert engine.verify_counts() == 0


@pytest.mark.parametrize("g", synth_goldens(), ids=lambda g: g["name"])
def test_synth_goldens_bit_exact(engine, g):
    m, c, st = _train(engine, synth_text(g), g["vocab_size"])
    assert m.tolist() == g["merges"]
    assert c.tolist() == g["counts"]
    assert st.final_tokens == g["final_tokens"]
    assert engine.verify_counts() == 0


@pytest.mark.parametrize("g", [g for g in synth_goldens() if g["n"] <= (1 << 18)], ids=lambda g: g["name"])
def test_tie_fast_path_agrees_with_exact_emulation(g):
    e = zbpe.Engine(0)
    e.set_option("exact_ties", 1)  # every tie also resolved by the exact emulation; mismatch -> error
    e.set_option("debug_checks", 1)
    m, c, st = e.train(synth_text(g), g["vocab_size"])
    assert m.tolist() == g["merges"]
    assert st.tie_fallbacks == st.tie_iterations
    e.close()


# --- the reference's inline tests (basic_tokenizer.zig:351-461) on the device ---------------------
def test_ref_train_hello(engine):
    t = zbpe.BasicTokenizer(engine=engine)
    t.train(b"hello world hello", 300, True)
    assert len(t.merges.merges) > 0
    enc = t.encode(b"hello")
    assert enc == [259]
    assert t.decode(enc) == b"hello"
    assert zbpe.merges_to_text(t.merges.as_array()) == O.serialize(O.train(b"hello world hello", 300).merges)


def test_ref_encode(engine):
    t = zbpe.BasicTokenizer(engine=engine)
    t.merges.put(zbpe.CharPair(ord("h"), ord("e")), 256)
    t.merges.put(zbpe.CharPair(256, ord("l")), 257)
    t.merges.put(zbpe.CharPair(ord("w"), ord("o")), 258)
    assert t.encode(b"hello world") == [257, ord("l"), ord("o"), ord(" "), 258, ord("r"), ord("l"), ord("d")]


def test_invalid_vocab(engine):
    with pytest.raises(zbpe.InvalidVocabSize):
        engine.train(b"abc", 255)


@pytest.mark.parametrize("text", [b"", b"a", b"ab", b"aa", b"aaa", b"aaaa", b"aaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaaa",
                                  b"abababababababababab", b"aabbaabbaaabbb", bytes(range(256)) * 3,
                                  b"\xff\xff\xff\x00\x00\xff", b"hello world hello"])
def test_edge_inputs(engine, text):
    vocab = 300
    r = O.train(text, vocab)
    m, c, st = _train(engine, text, vocab)
    assert m.tolist() == r.merges.tolist()
    assert c.tolist() == r.counts.tolist()
    assert st.final_tokens == len(r.tokens)


def test_vocab_256_no_merges(engine):
    m, c, st = _train(engine, b"hello", 256)
    assert len(m) == 0


@pytest.mark.parametrize("kind,n,vocab,seed", [("words", 50000, 700, 21), ("words_utf8", 200000, 800, 22),
                                               ("uniform", 20000, 600, 23), ("runs", 100000, 500, 24),
                                               ("runs", 7000, 800, 25), ("uniform", 1500, 2000, 26)])
def test_random_corpora_vs_oracle(engine, kind, n, vocab, seed):
    text = zbpe.synth_corpus(kind, seed, n)
    r = O.train(text, vocab)
    m, c, st = _train(engine, text, vocab)
    assert m.tolist() == r.merges.tolist()
    assert c.tolist() == r.counts.tolist()
    assert engine.verify_counts() == 0


@pytest.mark.parametrize("kind,n,vocab,seed", [("words_utf8", 2 << 20, 1500, 51), ("uniform", 1 << 16, 700, 52)])
def test_debug_checks_hot_list_and_compaction(kind, n, vocab, seed):
    """debug_checks: every merge cross-checks the hot-list argmax against a full argmax over all ids."""
    text = zbpe.synth_corpus(kind, seed, n)
    e = zbpe.Engine(0)
    e.set_option("debug_checks", 1)
    m, c, st = e.train(text, vocab)
    r = O.train(text, vocab, max_merges=300 if n > (1 << 20) else 0)
    assert m[: len(r.merges)].tolist() == r.merges.tolist()
    assert e.verify_counts() == 0
    e.close()


@pytest.mark.parametrize("g", synth_goldens(), ids=lambda g: g["name"])
@pytest.mark.parametrize("batch,skip,lists", [(1, 1, 1), (3, 0, 0), (256, 1, 1), (32, 1, 2), (1, 0, 2)])
def test_merge_batch_and_block_skip_agree(g, batch, skip, lists):
    """The synchronous loop (merge_batch 1), short and long device-resident batches (halting at self
    pairs, undecided ties and capacity changes), with and without block skipping and occurrence
    lists (2: lists from the first compaction on, every scan that can use one does): same merges."""
    e = zbpe.Engine(0)
    e.set_option("merge_batch", batch)
    e.set_option("block_skip", skip)
    e.set_option("list_mode", min(lists, 1))
    if lists == 2:
        e.set_option("list_start", 0)
        e.set_option("list_ratio", 1)
        e.set_option("compact_den", 2)
        e.set_option("compact_den_lists", 4)
    m, c, st = e.train(synth_text(g), g["vocab_size"])
    assert m.tolist() == g["merges"]
    assert c.tolist() == g["counts"]
    assert st.final_tokens == g["final_tokens"]
    assert e.verify_counts() == 0
    e.close()


def test_compaction_policies_agree(engine):
    text = zbpe.synth_corpus("words_utf8", 31, 300000)
    r = O.train(text, 700)
    for den in (1, 2, 64, 1 << 40):
        e = zbpe.Engine(0)
        e.set_option("compact_den", den)
        e.set_option("compact_den_lists", den)
        m, c, st = e.train(text, 700)
        assert m.tolist() == r.merges.tolist(), den
        assert e.verify_counts() == 0
        e.close()


def test_encode_vs_oracle(engine):
    text = zbpe.synth_corpus("words_utf8", 41, 400000)
    m, _, _ = _train(engine, text, 900)
    other = zbpe.synth_corpus("words_utf8", 42, 300000)
    for t in (text, other, b"", b"x"):
        assert np.array_equal(engine.encode(m, t), O.encode(m, t))


@pytest.mark.parametrize("list_mode,ratio", [(0, 256), (1, 1)])
def test_encode_list_and_stream_scans_vs_oracle(list_mode, ratio):
    """Encode with occurrence lists off, and on for every merge that can use one (ratio 1)."""
    e = zbpe.Engine(0)
    e.set_option("list_mode", list_mode)
    e.set_option("list_ratio", ratio)
    for kind, seed, n, vocab in (("words_utf8", 44, 300000, 800), ("runs", 45, 80000, 500), ("uniform", 46, 20000, 600)):
        text = zbpe.synth_corpus(kind, seed, n)
        m, _, _ = e.train(text, vocab)
        other = zbpe.synth_corpus(kind, seed + 100, n)
        for t in (text, other):
            assert np.array_equal(e.encode(m, t), O.encode(m, t)), (kind, list_mode)
    e.close()


@pytest.mark.parametrize("batch", [1, 2, 32])
def test_encode_batched_vs_oracle(batch):
    """Batched encode (disjoint consecutive merges applied together) equals the reference's merge-by-merge
    replay, with self pairs and merges sharing tokens breaking the batches."""
    e = zbpe.Engine(0)
    e.set_option("encode_batch", batch)
    for kind, seed, n, vocab in (("words_utf8", 47, 400000, 1200), ("runs", 48, 60000, 400), ("uniform", 49, 30000, 700)):
        text = zbpe.synth_corpus(kind, seed, n)
        m, _, _ = e.train(text, vocab)
        other = zbpe.synth_corpus(kind, seed + 100, n)
        for t in (text, other, text[:1], b""):
            assert np.array_equal(e.encode(m, t), O.encode(m, t)), (kind, batch)
        # a merge table whose order is shuffled within windows still encodes like the reference
        if kind == "words_utf8":
            rng = np.random.default_rng(seed)
            mm = m.copy()
            for s0 in range(0, len(mm) - 8, 8):
                mm[s0:s0 + 8] = mm[s0 + rng.permutation(8)]
            assert np.array_equal(e.encode(mm, other), O.encode(mm, other)), (kind, batch, "shuffled")
    e.close()


@pytest.mark.parametrize("self_batch", [0, 1])
@pytest.mark.parametrize("kind,seed,n,vocab", [("runs", 51, 60000, 500), ("words_utf8", 52, 300000, 900), ("uniform", 53, 8000, 700)])
def test_self_pairs_from_lists_vs_oracle(kind, seed, n, vocab, self_batch):
    """Self pairs (a, a) walked from a's occurrence list (lists built at the first compaction, used for
    every self pair) give the reference's merges and counts, in training and in encode -- on the host path
    (self_batch 0: every self pair halts its batch) and inside the device's batches (self_batch 1)."""
    text = zbpe.synth_corpus(kind, seed, n)
    r = O.train(text, vocab)
    e = zbpe.Engine(0)
    e.set_option("self_batch", self_batch)
    e.set_option("list_start", 0)
    e.set_option("compact_den", 2)
    e.set_option("compact_den_lists", 2)
    e.set_option("self_list_ratio", 1)
    m, c, st = e.train(text, vocab)
    assert m.tolist() == r.merges.tolist()
    assert c.tolist() == r.counts.tolist()
    assert e.verify_counts() == 0
    e.set_option("list_ratio", 1)
    other = zbpe.synth_corpus(kind, seed + 100, n)
    for t in (text, other):
        assert np.array_equal(e.encode(m, t), O.encode(m, t))
    e.close()


@pytest.mark.parametrize("encode_batch", [1, 32])
def test_encode_new_token_equals_first_vs_oracle(encode_batch):
    """A merge table (e.g. from deserializeMerges) may hold (a, b) -> a. The reference's encode re-tests
    position i after merging there (basic_tokenizer.zig:71-88 does not advance i), so a absorbs the whole
    run of b's after it, and (a, a) -> a collapses a run of a's: the device repeats such a merge until a
    pass finds no occurrence. Compared with the oracle's literal orderedRemove loop."""
    e = zbpe.Engine(0)
    e.set_option("encode_batch", encode_batch)
    text = zbpe.synth_corpus("runs", 54, 50000) + b"abbbbbab aaaaaaa bbbb abab" * 50
    m, _, _ = e.train(text, 400)
    a, b = ord("a"), ord("b")
    x = int(m[0][2])
    tables = [
        np.array([[a, b, a]], dtype=np.uint16),                       # a absorbs runs of b
        np.array([[a, a, a]], dtype=np.uint16),                       # runs of a collapse
        np.array([[b, b, b], [a, b, a]], dtype=np.uint16),
        np.concatenate([m[:20], np.array([[x, a, x], [a, b, a]], dtype=np.uint16), m[20:40]]),
    ]
    for mm in tables:
        for t in (text, b"ab", b"abb", b"aab", b"bbbb", b"", text[:997]):
            assert np.array_equal(e.encode(mm, t), O.encode(mm, t, literal=True)), (mm[:3].tolist(), t[:20])
    e.close()


def test_encode_runs_vs_oracle(engine):
    text = zbpe.synth_corpus("runs", 43, 100000)
    m, _, _ = _train(engine, text, 600)
    assert np.array_equal(engine.encode(m, text), O.encode(m, text))


def test_oracle_prefix_first_merges_large(engine):
    """At 16 MiB the oracle can still run a few merges: the first merges must agree."""
    text = zbpe.synth_corpus("words", 77, 16 << 20)
    r = O.train(text, 262)
    m, c, st = _train(engine, text, 262)
    assert m.tolist() == r.merges.tolist()
    assert c.tolist() == r.counts.tolist()


def test_c_abi_consumer_mirrors_main_zig(tmp_path):
    """tests/c_abi/main (C, include/zbpe.h + libzbpe.so only) does what src/main.zig:8-43 does: train
    taylorswift.txt at vocab 300, write merges.txt, encode and decode the main.zig:25 string. merges.txt
    must be the reference's bytes and decode(encode(s)) == s; the tokens equal the oracle's encode."""
    import os
    import subprocess

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    exe = os.path.join(root, "tests", "c_abi", "main")
    assert os.access(exe, os.X_OK), "tests/c_abi/main not built (__graft_entry__.build())"
    txt = tmp_path / "taylorswift.txt"
    txt.write_bytes(c1_text())
    out = tmp_path / "merges.txt"
    r = subprocess.run([exe, str(txt), str(out)], capture_output=True, timeout=120)
    assert r.returncode == 0, r.stderr.decode(errors="replace")
    assert out.read_bytes() == c1_merges_txt()
    msg = "hello world!!!? (안녕하세요!) lol123 😉".encode()
    lines = r.stdout.decode().splitlines()
    want = O.encode(np.asarray(c1_golden()["merges"], dtype=np.uint16), msg)
    assert lines[1].split() == [str(int(t)) for t in want]
    assert lines[2].encode() == msg
    assert b"Time statistics:" in r.stderr and b"sortCodePointPairs:" in r.stderr


def test_verbose_lines_match_print_merge_info(capfd):
    """verbose=True prints printMergeInfo's line per merge (basic_tokenizer.zig:308-317), identical to
    the oracle's, in merge order (the device-resident batches print theirs after each batch)."""
    text = c1_text()
    e = zbpe.Engine(0)
    capfd.readouterr()
    O.train(text, 300, verbose=True)
    ref = [l for l in capfd.readouterr().err.splitlines() if l.startswith("merge ")]
    e.train(text, 300, verbose=True)
    got = [l for l in capfd.readouterr().err.splitlines() if l.startswith("merge ")]
    e.close()
    assert len(ref) == 44 and got == ref
    text = synth_text(synth_goldens()[0])
    e = zbpe.Engine(0)
    O.train(text, 400, verbose=True)
    ref = [l for l in capfd.readouterr().err.splitlines() if l.startswith("merge ")]
    e.train(text, 400, verbose=True)
    got = [l for l in capfd.readouterr().err.splitlines() if l.startswith("merge ")]
    e.close()
    assert got == ref


def test_basic_tokenizer_prints_time_stats(capfd):
    """BasicTokenizer.train prints printTimeStats' block at its end, like the reference's defer (:141-145);
    the GPU buckets never exceed the call's wall time."""
    t = zbpe.BasicTokenizer()
    capfd.readouterr()
    t.train(c1_text(), 300)
    err = capfd.readouterr().err
    for name in ("sortCodePointPairs", "replaceTopPairWithIndex", "generateCodePointPairs", "countPointPairs",
                 "Other operations"):
        assert name + ":" in err
    st = t.timeStats
    assert st.count_pairs_s + st.sort_pairs_s + st.replace_pair_s <= st.total_s + 1e-6
    assert st.replace_pair_calls == 44 and st.sort_pairs_calls >= 44
    t.deinit()


@pytest.mark.parametrize("cap", [2000, 50000])
def test_small_arena_grows_and_matches_oracle(cap):
    """A shrunken occurrence arena (option arena_cap): compactions and growth of the arena (keeping its
    lists) when a merge needs more room; merges and counts still equal the oracle's."""
    text = zbpe.synth_corpus("words_utf8", 71, 200000)
    r = O.train(text, 700)
    e = zbpe.Engine(0)
    e.set_option("arena_cap", cap)
    e.set_option("list_start", 0)
    m, c, st = e.train(text, 700)
    assert m.tolist() == r.merges.tolist() and c.tolist() == r.counts.tolist()
    assert e.verify_counts() == 0
    e.close()


@pytest.mark.parametrize("nb", [0, 1])
def test_list_neighbour_filter_agrees(nb):
    """List scans with and without the build-time neighbour filter (option list_nb) give the oracle's
    merges, with lists from the first compaction on and every scan that can use one walking it."""
    for kind, seed, n, vocab in (("words_utf8", 72, 300000, 900), ("runs", 73, 60000, 500), ("uniform", 74, 20000, 700)):
        text = zbpe.synth_corpus(kind, seed, n)
        r = O.train(text, vocab)
        e = zbpe.Engine(0)
        e.set_option("list_nb", nb)
        e.set_option("list_start", 0)
        e.set_option("list_ratio", 1)
        e.set_option("compact_den", 2)
        m, c, st = e.train(text, vocab)
        assert m.tolist() == r.merges.tolist() and c.tolist() == r.counts.tolist(), (kind, nb)
        assert e.verify_counts() == 0
        other = zbpe.synth_corpus(kind, seed + 100, n)
        assert np.array_equal(e.encode(m, other), O.encode(m, other)), (kind, nb)
        e.close()


def test_encode_table_with_token_65535():
    """deserializeMerges accepts any u16 (basic_tokenizer.zig:342-344), so a table may create or use token
    65535 (the device's hole marker): encode renames it internally and must equal the reference's loop"""
    text = synth_text(synth_goldens()[0])[:50000]
    tables = [
        [(101, 32, 65535), (65535, 116, 300), (116, 104, 301)],
        [(32, 116, 65535), (104, 101, 300), (65535, 300, 301), (65535, 65535, 302)],
        [(65535, 97, 256), (97, 98, 257)],  # a merge on a token nothing produces
    ]
    e = zbpe.Engine(0)
    for tab in tables:
        m = np.asarray(tab, dtype=np.uint16)
        assert e.encode(m, text).tolist() == O.encode(m, text, literal=True).tolist()
    e.close()


def test_generate_initial_tokens_runtime_line(capfd):
    """train and encode print generateInitialTokens' runtime line like the reference (:156-160, called by
    train :150 and encode :72)"""
    e = zbpe.Engine(0)
    capfd.readouterr()
    m, _, st = e.train(b"hello world hello", 300)
    err = capfd.readouterr().err
    assert err.count("generateInitialTokens runtime: ") == 1 and " seconds\n" in err and st.generate_tokens_s >= 0
    e.encode(m, b"hello")
    assert capfd.readouterr().err.startswith("generateInitialTokens runtime: ")
    e.set_option("print_runtime", 0)
    e.train(b"hello world hello", 300)
    assert "generateInitialTokens" not in capfd.readouterr().err
    e.close()


def test_basic_tokenizer_time_stats_accumulate(capfd):
    """TimeStats live as long as the tokenizer (time_statistics.zig:15-29): a second train adds to them"""
    t = zbpe.BasicTokenizer()
    t.train(c1_text(), 300)
    calls = t.timeStats.replace_pair_calls
    t.train(c1_text(), 300)
    assert t.timeStats.replace_pair_calls == 2 * calls == 88
    assert len(t.merges.merges) == 88  # merges append (:199)
    t.deinit()


@pytest.mark.parametrize("variant,batch", [(v, 1) for v in range(7)] + [(7, 0), (7, 2)])
@pytest.mark.parametrize("kind,n,vocab,seed", [("words_utf8", 300000, 900, 61), ("runs", 60000, 600, 62)])
def test_scan_variants_agree_with_oracle(variant, batch, kind, n, vocab, seed):
    """Every stream-form scan variant (engine.hip kScanVariants; 7 with cross-tile candidate batching
    off / always) on streams with holes, lists off so every merge streams: oracle merges and counts."""
    text = zbpe.synth_corpus(kind, seed, n)
    r = O.train(text, vocab)
    for merge_batch, skip in ((1, 0), (64, 1)):
        e = zbpe.Engine(0)
        e.set_option("scan_variant", variant)
        e.set_option("scan_batch", batch)
        e.set_option("list_mode", 0)
        e.set_option("compact_den", 1 << 40)  # holes stay: windows and hole runs in the resolve paths
        e.set_option("merge_batch", merge_batch)
        e.set_option("block_skip", skip)
        m, c, st = e.train(text, vocab)
        assert m.tolist() == r.merges.tolist(), (merge_batch, skip)
        assert c.tolist() == r.counts.tolist(), (merge_batch, skip)
        assert e.verify_counts() == 0
        e.close()


def test_scan_batch_option_range(engine):
    with pytest.raises(zbpe.ZbpeError):
        engine.set_option("scan_batch", 3)


@pytest.mark.parametrize("min_len,max_rows", [(1, 65536), (64, 8), (1 << 30, 4096)], ids=["all_lists", "few_rows", "none"])
def test_list_successor_ranges_agree(min_len, max_rows):
    """Successor-sorted long lists (options list_ranges, range_min_len, range_max_rows): a scan of two
    pre-build tokens walks only a's entries whose build-time successor was b. Every list sorted, a few
    rows, or none: the oracle's merges and counts; the merge log shows range walks of ~count entries."""
    for kind, seed, n, vocab in (("words_utf8", 75, 400000, 1000), ("runs", 76, 60000, 500), ("uniform", 77, 30000, 700)):
        text = zbpe.synth_corpus(kind, seed, n)
        r = O.train(text, vocab)
        for merge_batch in (1, 64):
            e = zbpe.Engine(0)
            e.set_option("list_start", 0)
            e.set_option("list_ratio", 1)
            e.set_option("compact_den", 2)
            e.set_option("range_min_len", min_len)
            e.set_option("range_max_rows", max_rows)
            e.set_option("merge_batch", merge_batch)
            m, c, st = e.train(text, vocab)
            assert m.tolist() == r.merges.tolist() and c.tolist() == r.counts.tolist(), (kind, merge_batch)
            assert e.verify_counts() == 0
            L = e.merge_log()
            ranged = L[:, 7] == 1
            if min_len == 1 and merge_batch == 64 and kind == "words_utf8":
                assert ranged.sum() > 0, kind
                # a range holds the pair's occurrences at the build, so at least its count
                assert np.all(L[ranged, 5] >= L[ranged, 1]), kind
            if min_len == 1 << 30:
                assert ranged.sum() == 0
            e.close()


def test_list_ranges_on_c2_bit_exact():
    g = [x for x in synth_goldens() if x["n"] >= (1 << 20)]
    for gg in g[:1]:
        e = zbpe.Engine(0)
        e.set_option("list_start", 0)
        e.set_option("range_min_len", 256)
        m, c, st = e.train(synth_text(gg), gg["vocab_size"])
        assert m.tolist() == gg["merges"] and c.tolist() == gg["counts"]
        e.close()


@pytest.mark.parametrize("kind", ["abac", "c4_slice", "utf8", "sharded_tail"])
def test_pair_hist_bytes_exact(kind):
    """The full pair histogram of a byte stream (zbpe_pair_hist_bytes: every byte pair in a fixed 16-bit LDS
    bin, overflow accounted from the adds' return values) equals the incremental table at t = 0 (verify_counts
    after training zero merges) and the hashed form's result. 'abac' repeated puts ~100 K adds of (a,b) and
    (a,c) -- the two halves of ONE word -- into every workgroup: both halves wrap, and the low half's carry
    is taken back while the high half is being added to."""
    if kind == "abac":
        text = b"abac" * (24 << 20)
    elif kind == "c4_slice":
        text = zbpe.synth_corpus("words_utf8", 0x5EED0004, 96 << 20, threads=16)
    elif kind == "utf8":
        text = bytes(range(256)) * 4096 + zbpe.synth_corpus("uniform", 5, 1 << 20)
    else:
        text = b"ab" * 1000 + b"x"  # an odd length: the last vector's tail pairs
    e = zbpe.Engine(0)
    try:
        e.upload(text)
        for dense in (1, 0):
            e.set_option("dense_hist", dense)
            e.train_resident(256)
            assert e.verify_counts() == 0, dense
            r = e.bench_recount(1)
            assert r["mismatches"] == 0 and r["tokens"] == len(text)
    finally:
        e.close()
