"""TEST INFRASTRUCTURE ONLY -- ctypes loader for the CPU oracle (oracle/zig_ref.c).

The oracle restates /root/reference/src/basic_tokenizer.zig (train :140-306, encode :71-88,
decode :90-138, serializeMerges :319-330) plus the Zig 0.13 std semantics that decide the
tie-break (Wyhash seed 0, HashMapUnmanaged slot order, stable block sort).  Only tests/,
__graft_entry__.smoke() and bench.py's cpu_baseline leg import this module; the product
(zig-bpe_amd/) never does.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from dataclasses import dataclass
from typing import Optional

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = os.path.join(_HERE, "libzref.so")


class ZrefStats(ctypes.Structure):
    _fields_ = [
        ("sort_pairs_s", ctypes.c_double),
        ("replace_pair_s", ctypes.c_double),
        ("generate_pairs_s", ctypes.c_double),
        ("count_pairs_s", ctypes.c_double),
        ("total_s", ctypes.c_double),
        ("sort_pairs_calls", ctypes.c_uint64),
        ("replace_pair_calls", ctypes.c_uint64),
        ("generate_pairs_calls", ctypes.c_uint64),
        ("count_pairs_calls", ctypes.c_uint64),
        ("pair_tokens", ctypes.c_uint64),
        ("tie_iterations", ctypes.c_uint64),
    ]


def build() -> str:
    if not os.path.exists(_LIB) or os.path.getmtime(_LIB) < os.path.getmtime(os.path.join(_HERE, "zig_ref.c")):
        subprocess.run(["make", "-s", "-C", _HERE, "libzref.so"], check=True)
    return _LIB


_lib = None


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        L = ctypes.CDLL(build())
        L.zref_wyhash.restype = ctypes.c_uint64
        L.zref_wyhash.argtypes = [ctypes.c_uint64, ctypes.c_char_p, ctypes.c_size_t]
        L.zref_pair_hash.restype = ctypes.c_uint64
        L.zref_pair_hash.argtypes = [ctypes.c_uint16, ctypes.c_uint16]
        L.zref_selftest.restype = ctypes.c_int
        L.zref_train.restype = ctypes.c_int
        L.zref_map_order.restype = ctypes.c_uint32
        L.zref_encode.restype = ctypes.c_int
        L.zref_decode.restype = ctypes.c_int
        L.zref_step.restype = ctypes.c_int
        L.zref_train_log.restype = ctypes.c_int
        L.zref_fnv64.restype = ctypes.c_uint64
        _lib = L
    return _lib


def _p(a: np.ndarray):
    return a.ctypes.data_as(ctypes.c_void_p)


@dataclass
class TrainResult:
    merges: np.ndarray      # (M, 3) uint16: first, second, new_token
    counts: np.ndarray      # (M,) uint64 top count per merge
    ties: np.ndarray        # (M,) uint32 pairs sharing the top count
    distinct: np.ndarray    # (M,) uint32 distinct pairs D_t
    tokens: np.ndarray      # final token stream (uint16)
    stats: ZrefStats


def train(text: bytes, vocab_size: int, verbose: bool = False, max_merges: int = 0) -> TrainResult:
    L = lib()
    cap = max(vocab_size - 256, 0)
    tri = np.zeros(3 * max(cap, 1), dtype=np.uint16)
    cnt = np.zeros(max(cap, 1), dtype=np.uint64)
    ties = np.zeros(max(cap, 1), dtype=np.uint32)
    dist = np.zeros(max(cap, 1), dtype=np.uint32)
    toks = np.zeros(max(len(text), 1), dtype=np.uint16)
    nm = ctypes.c_size_t(0)
    nt = ctypes.c_size_t(0)
    st = ZrefStats()
    buf = np.frombuffer(text, dtype=np.uint8) if len(text) else np.zeros(1, dtype=np.uint8)
    rc = L.zref_train(_p(buf), ctypes.c_size_t(len(text)), ctypes.c_uint32(vocab_size), ctypes.c_int(int(verbose)),
                      ctypes.c_uint32(max_merges), _p(tri), _p(cnt), _p(ties), _p(dist), ctypes.byref(nm),
                      ctypes.byref(st), _p(toks), ctypes.byref(nt))
    if rc == 1:
        raise ValueError("InvalidVocabSize")
    if rc != 0:
        raise MemoryError("OutOfMemory")
    m = nm.value
    return TrainResult(tri[: 3 * m].reshape(m, 3).copy(), cnt[:m].copy(), ties[:m].copy(), dist[:m].copy(),
                       toks[: nt.value].copy(), st)


@dataclass
class StepResult:
    pair: tuple        # (first, second) of sortedCodePointPairs[0]
    count: int         # its count
    ties: int          # pairs sharing that count
    distinct: int      # D_t: distinct pairs of the stream
    stats: ZrefStats


def step(tokens, literal: bool = False) -> Optional[StepResult]:
    """One expandVocabulary iteration (basic_tokenizer.zig:183-204) on a u16 token stream: the pair
    the reference would merge next. None when the stream has no pairs (:188-191)."""
    L = lib()
    t = np.ascontiguousarray(np.asarray(tokens, dtype=np.uint16))
    tt = t if len(t) else np.zeros(1, dtype=np.uint16)
    pair, cnt, ties, d = ctypes.c_uint32(0), ctypes.c_uint64(0), ctypes.c_uint32(0), ctypes.c_uint64(0)
    st = ZrefStats()
    rc = L.zref_step(_p(tt), ctypes.c_size_t(len(t)), ctypes.c_int(int(literal)), ctypes.byref(pair), ctypes.byref(cnt),
                     ctypes.byref(ties), ctypes.byref(d), ctypes.byref(st))
    if rc == 3:
        return None
    if rc != 0:
        raise MemoryError("OutOfMemory")
    return StepResult((pair.value & 0xFFFF, pair.value >> 16), int(cnt.value), int(ties.value), int(d.value), st)


def map_order(tokens) -> tuple[np.ndarray, np.ndarray, np.ndarray, int]:
    """Slot-ordered (keys, slots, counts) of the Zig pair map built from `tokens`, and its capacity."""
    L = lib()
    t = np.ascontiguousarray(np.asarray(tokens, dtype=np.uint16))
    n = len(t)
    k = np.zeros(max(n, 1), dtype=np.uint32)
    s = np.zeros(max(n, 1), dtype=np.uint32)
    c = np.zeros(max(n, 1), dtype=np.uint64)
    d = ctypes.c_size_t(0)
    tt = t if n else np.zeros(1, dtype=np.uint16)
    cap = L.zref_map_order(_p(tt), ctypes.c_size_t(n), _p(k), _p(s), _p(c), ctypes.byref(d))
    d = d.value
    return k[:d].copy(), s[:d].copy(), c[:d].copy(), int(cap)


def encode(merges: np.ndarray, text: bytes, literal: bool = False) -> np.ndarray:
    L = lib()
    tri = np.ascontiguousarray(np.asarray(merges, dtype=np.uint16).reshape(-1))
    out = np.zeros(max(len(text), 1), dtype=np.uint16)
    n = ctypes.c_size_t(0)
    buf = np.frombuffer(text, dtype=np.uint8) if len(text) else np.zeros(1, dtype=np.uint8)
    tri_p = tri if len(tri) else np.zeros(3, dtype=np.uint16)
    L.zref_encode(_p(tri_p), ctypes.c_size_t(len(tri) // 3), _p(buf), ctypes.c_size_t(len(text)),
                  ctypes.c_int(int(literal)), _p(out), ctypes.byref(n))
    return out[: n.value].copy()


def decode(merges: np.ndarray, tokens) -> bytes:
    L = lib()
    tri = np.ascontiguousarray(np.asarray(merges, dtype=np.uint16).reshape(-1))
    t = np.ascontiguousarray(np.asarray(tokens, dtype=np.uint16))
    cap = 1 << 20
    while True:
        out = np.zeros(cap, dtype=np.uint8)
        n = ctypes.c_size_t(0)
        tri_p = tri if len(tri) else np.zeros(3, dtype=np.uint16)
        tp = t if len(t) else np.zeros(1, dtype=np.uint16)
        rc = L.zref_decode(_p(tri_p), ctypes.c_size_t(len(tri) // 3), _p(tp), ctypes.c_size_t(len(t)), _p(out),
                           ctypes.c_size_t(cap), ctypes.byref(n))
        if rc == 2:
            cap *= 8
            continue
        if rc == 1:
            raise ValueError("InvalidToken")
        return out[: n.value].tobytes()


def serialize(merges: np.ndarray) -> bytes:
    """serializeMerges (basic_tokenizer.zig:319-330): "{first},{second},{new_token}\\n" per merge."""
    return "".join(f"{int(a)},{int(b)},{int(c)}\n" for a, b, c in np.asarray(merges).reshape(-1, 3)).encode()


def fnv64(tokens) -> int:
    """FNV-1a 64 of a u16 token stream's little-endian bytes (the long-run goldens' stream checksum)."""
    t = np.ascontiguousarray(np.asarray(tokens, dtype=np.uint16))
    tt = t if len(t) else np.zeros(1, dtype=np.uint16)
    return int(lib().zref_fnv64(_p(tt), ctypes.c_size_t(len(t))))


_FAST = os.path.join(_HERE, "libzfast.so")
_fast = None


def fast_lib() -> ctypes.CDLL:
    """oracle/zig_fast.cpp: the second restatement (incremental counts + a literal Zig-map replay at
    every tied merge), fast enough for C4 in full."""
    global _fast
    if _fast is None:
        src = os.path.join(_HERE, "zig_fast.cpp")
        if not os.path.exists(_FAST) or os.path.getmtime(_FAST) < os.path.getmtime(src):
            subprocess.run(["make", "-s", "-C", _HERE, "libzfast.so"], check=True)
        L = ctypes.CDLL(_FAST)
        L.zfast_train.restype = ctypes.c_int
        L.zfast_pair_hash.restype = ctypes.c_uint64
        L.zfast_pair_hash.argtypes = [ctypes.c_uint32]
        L.zfast_final_capacity.restype = ctypes.c_uint32
        L.zfast_final_capacity.argtypes = [ctypes.c_uint64, ctypes.c_int]
        _fast = L
    return _fast


@dataclass
class FastResult:
    merges: np.ndarray      # (M, 3) uint16
    counts: np.ndarray      # (M,) uint64
    ties: np.ndarray        # (M,) uint32
    distinct: np.ndarray    # (M,) uint32
    len_after: np.ndarray   # (M,) uint64 stream length after each merge
    tokens: np.ndarray      # final stream
    restarts: int           # runs restarted because a replay overruled a predicted winner
    ties_sync: int          # tied merges replayed before the merge
    ties_async: int         # tied merges replayed by the worker threads (and confirmed)


def fast_train(text: bytes, vocab_size: int, threads: int = 4, sync_limit: int = 1 << 20, fnv_every: int = 0,
               progress: Optional[str] = None) -> FastResult:
    L = fast_lib()
    cap = max(vocab_size - 256, 1)
    n = len(text)
    tri = np.zeros(3 * cap, np.uint16)
    cnt = np.zeros(cap, np.uint64)
    ties = np.zeros(cap, np.uint32)
    dist = np.zeros(cap, np.uint32)
    lens = np.zeros(cap, np.uint64)
    fin = np.zeros(max(n, 1), np.uint16)
    info = np.zeros(4, np.uint64)
    nm, nf = ctypes.c_size_t(0), ctypes.c_size_t(0)
    buf = np.frombuffer(text, np.uint8) if n else np.zeros(1, np.uint8)
    rc = L.zfast_train(_p(buf), ctypes.c_size_t(n), ctypes.c_uint32(vocab_size), ctypes.c_int(threads),
                       ctypes.c_uint64(sync_limit), ctypes.c_uint32(fnv_every),
                       progress.encode() if progress else None, _p(tri), _p(cnt), _p(ties), _p(dist), _p(lens),
                       ctypes.byref(nm), _p(fin), ctypes.byref(nf), _p(info))
    if rc == 1:
        raise ValueError("InvalidVocabSize")
    if rc != 0:
        raise MemoryError(f"zfast_train rc {rc}")
    m = nm.value
    return FastResult(tri[: 3 * m].reshape(m, 3).copy(), cnt[:m].copy(), ties[:m].copy(), dist[:m].copy(),
                      lens[:m].copy(), fin[: nf.value].copy(), int(info[0]), int(info[1]), int(info[2]))


def wyhash(seed: int, data: bytes) -> int:
    return int(lib().zref_wyhash(ctypes.c_uint64(seed), data, ctypes.c_size_t(len(data))))


def pair_hash(first: int, second: int) -> int:
    return int(lib().zref_pair_hash(ctypes.c_uint16(first), ctypes.c_uint16(second)))


def selftest() -> int:
    return int(lib().zref_selftest())
