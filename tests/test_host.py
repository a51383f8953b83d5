"""CPU tests of the product's host side: the C ABI library loads and exports every symbol the
header declares, the host Zig-order emulator, the BasicTokenizer mirror's host methods
(decode / serializeMerges / deserializeMerges, basic_tokenizer.zig:90-138,319-348)."""
import os
import re

import numpy as np
import pytest

import oracle as O
import zbpe
from conftest import ROOT, gpu_available
from helpers import c1_text, synth_goldens, synth_text


def test_library_exports_header_symbols():
    L = zbpe.load_library()
    hdr = open(os.path.join(ROOT, "include", "zbpe.h")).read()
    names = set(re.findall(r"\b(zbpe_[a-z_0-9]+)\s*\(", hdr))
    assert names == set(zbpe.EXPORTS)
    for n in names:
        assert hasattr(L, n), n
    assert L.zbpe_version().startswith(b"zbpe-mi355x")


@pytest.mark.skipif(gpu_available(), reason="only meaningful without a GPU")
def test_no_cpu_fallback_without_gpu():
    with pytest.raises(zbpe.DeviceError):
        zbpe.Engine(0)


def _zig_check(tokens):
    keys, slots, counts, cap = O.map_order(tokens)
    if len(keys) == 0:
        return
    first = {}
    for i in range(len(tokens) - 1):
        first.setdefault(int(tokens[i]) | (int(tokens[i + 1]) << 16), i)
    fp = [first[int(k)] for k in keys]
    last = int(tokens[-2]) | (int(tokens[-1]) << 16)
    call_after = int(counts[list(keys).index(last)]) >= 2
    for top in sorted(set(int(c) for c in counts))[-3:]:
        want = int(keys[[i for i, c in enumerate(counts) if c == top][0]])
        # shuffle the input order: the emulator must sort by first occurrence itself
        perm = np.random.default_rng(top).permutation(len(keys))
        got = zbpe.zig_order_winner(np.array(fp)[perm], keys[perm], counts[perm].astype(np.uint32), top, call_after)
        assert got == want


def test_zig_order_emulator_matches_oracle():
    _zig_check(list(b"hello world hello"))
    _zig_check(list(c1_text()))
    for g in synth_goldens():
        if g["n"] <= (1 << 16):
            r = O.train(synth_text(g), min(g["vocab_size"], 300))
            _zig_check(r.tokens)


@pytest.mark.parametrize("threads", [2, 4, 8, 16])
def test_zig_order_parallel_levels_match(monkeypatch, threads):
    """The parallel level builder (segments cut at slots empty in the final table, zig_order.hpp) gives the
    same Zig order as the one-thread replay: real streams against the oracle's map (every level parallel),
    and random live sets with many ties, each winner checked against the sequential build."""
    monkeypatch.setenv("ZBPE_EMU_THREADS", str(threads))
    monkeypatch.setenv("ZBPE_EMU_PAR_MIN", "0")
    _zig_check(list(c1_text()))
    g = [x for x in synth_goldens() if x["kind"] == "words_utf8"][0]
    _zig_check(O.train(synth_text(g), 300).tokens)
    rng = np.random.default_rng(threads)
    for n, call_after in ((5000, False), (200000, True), (419430, False), (419430, True)):  # 419430 = max load of 2^19
        keys = rng.choice(1 << 31, size=n, replace=False).astype(np.uint32)
        first = rng.permutation(n).astype(np.uint32)
        counts = rng.integers(1, 40, size=n).astype(np.uint32)
        top = 39
        monkeypatch.setenv("ZBPE_EMU_PAR_MIN", "0")
        par = zbpe.zig_order_winner(first, keys, counts, top, call_after)
        monkeypatch.setenv("ZBPE_EMU_PAR_MIN", str(1 << 40))
        seq = zbpe.zig_order_winner(first, keys, counts, top, call_after)
        assert par == seq


def test_zig_order_parallel_level_tables_equal(tmp_path):
    """tests/model/zig_emu_check.cpp: the parallel level builder's table equals the one-thread replay's,
    slot for slot (random sequences, loads 30-80 %, 2-16 threads)"""
    import subprocess

    exe = tmp_path / "zig_emu_check"
    src = os.path.join(ROOT, "tests", "model", "zig_emu_check.cpp")
    subprocess.run(["g++", "-O2", "-std=c++17", "-pthread", "-o", str(exe), src], check=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr


def test_synth_corpus_deterministic():
    a = zbpe.synth_corpus("words_utf8", 5, 3 << 20, threads=1)
    b = zbpe.synth_corpus("words_utf8", 5, 3 << 20, threads=7)
    assert a == b
    assert zbpe.synth_corpus("words", 5, 1000) != zbpe.synth_corpus("words", 6, 1000)
    u = np.frombuffer(zbpe.synth_corpus("words_utf8", 5, 1 << 20), np.uint8)
    assert 0.01 < (u >= 128).mean() < 0.2


def _tok_with(merges):
    t = zbpe.BasicTokenizer()
    for a, b, c in merges:
        t.merges.put(zbpe.CharPair(a, b), c)
    return t


def test_decode_reference_case_and_errors():
    t = _tok_with([(104, 101, 256), (256, 108, 257), (119, 111, 258)])
    assert t.decode([257, 108, 111, 32, 258, 114, 108, 100]) == b"hello world"
    with pytest.raises(zbpe.InvalidToken):
        t.decode([259])
    # findMerge returns the FIRST merge with that new_token (:109-116)
    t2 = _tok_with([(97, 98, 256), (99, 100, 256)])
    assert t2.decode([256]) == b"ab"
    # unknown sub-token inside a merge
    with pytest.raises(zbpe.InvalidToken):
        _tok_with([(300, 97, 256)]).decode([256])


def test_decode_matches_oracle():
    r = O.train(c1_text(), 300)
    t = _tok_with([tuple(int(x) for x in m) for m in r.merges])
    assert t.decode(r.tokens) == c1_text()
    assert t.decode(r.tokens) == O.decode(r.merges, r.tokens)


def test_serialize_format(tmp_path):
    t = _tok_with([(101, 32, 256), (44, 32, 257)])
    p = tmp_path / "m.txt"
    t.serializeMerges(str(p))
    assert p.read_bytes() == b"101,32,256\n44,32,257\n"


@pytest.mark.parametrize("content,err", [
    (b"1,2\n", zbpe.InvalidFormat),
    (b"1\n", zbpe.InvalidFormat),
    (b"1,2,70000\n", zbpe.Overflow),
    (b"1,2,3\r\n", zbpe.InvalidCharacter),
    (b"\n", zbpe.InvalidCharacter),
    (b"1,2,x\n", zbpe.InvalidCharacter),
    (b"1,2,-1\n", zbpe.Overflow),
    (b"1,2," + b"0" * 96 + b"3\n", zbpe.StreamTooLong),
])
def test_deserialize_errors(tmp_path, content, err):
    p = tmp_path / "m.txt"
    p.write_bytes(content)
    with pytest.raises(err):
        zbpe.BasicTokenizer().deserializeMerges(str(p))


def test_deserialize_semantics(tmp_path):
    p = tmp_path / "m.txt"
    # 99 content bytes + newline fit the 100-byte buffer; last line may lack a newline; extra fields ignored
    long_ok = b"1,2," + b"0" * 92 + b"3"
    assert len(long_ok) == 97
    p.write_bytes(b"1,2,256\n+3,4_0,2_57,9\n" + long_ok + b"\n5,6,-0")
    t = _tok_with([(9, 9, 300)])
    t.deserializeMerges(str(p))  # appends (:346)
    got = [(m.pair.first, m.pair.second, m.new_token) for m in t.merges.merges]
    assert got == [(9, 9, 300), (1, 2, 256), (3, 40, 257), (1, 2, 3), (5, 6, 0)]


def test_c_abi_consumer_builds():
    """tests/c_abi/main.c includes only include/zbpe.h and links only libzbpe.so: the header compiles
    as C11 (-pedantic -Werror) and C++17, and every entry point main.zig's flow needs resolves."""
    import subprocess
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    subprocess.run(["make", "-s", "-C", os.path.join(root, "tests", "c_abi")], check=True)
    assert os.access(os.path.join(root, "tests", "c_abi", "main"), os.X_OK)


def test_time_stats_printed_on_invalid_vocab(capfd):
    """printTimeStats runs from train's defer (basic_tokenizer.zig:141-145), so it prints on
    InvalidVocabSize too (no device work happens before the check)"""
    t = zbpe.BasicTokenizer()
    capfd.readouterr()
    with pytest.raises(zbpe.InvalidVocabSize):
        t.train(b"abc", 100)
    err = capfd.readouterr().err
    assert "Time statistics:" in err and "sortCodePointPairs: 0.000s total, 0 calls, nans avg" in err
