"""zbpe -- MI355X BPE trainer behind zig-bpe's BasicTokenizer API.

Mirrors /root/reference/src/basic_tokenizer.zig:
  BasicTokenizer.init / deinit            (:57-69)
  BasicTokenizer.train(text, vocabSize, verbose)   (:140-153)   -> libzbpe.so zbpe_train (HIP)
  BasicTokenizer.encode(text)              (:71-88)    -> libzbpe.so zbpe_encode (HIP)
  BasicTokenizer.decode(tokens)            (:90-138)   host (boundary API, no device work)
  BasicTokenizer.serializeMerges(path)     (:319-330)  host
  BasicTokenizer.deserializeMerges(path)   (:332-348)  host
  tokenizer.merges.merges[i].pair.first / .second / .new_token, tokenizer.merges.put(pair, tok)
Error names follow the reference (TrainError.{InvalidVocabSize, InvalidUtf8, OutOfMemory},
error.InvalidToken, error.InvalidFormat, std.fmt.parseInt's Overflow/InvalidCharacter,
readUntilDelimiterOrEof's StreamTooLong).

The device path is the only path: if libzbpe.so is missing or no GPU is present, train/encode
raise; nothing falls back to a CPU implementation.
"""
from __future__ import annotations

import ctypes
import os
import sys
import time
from dataclasses import dataclass, field
from typing import Iterable, List, Optional, Sequence

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("ZBPE_LIB") or os.path.join(_HERE, "libzbpe.so")  # ZBPE_LIB: A/B of builds
SYNTH_PATH = os.path.join(_HERE, "libzbpe_synth.so")

vocabStart = 256  # basic_tokenizer.zig:50

# ---------------------------------------------------------------------------------------------
# errors (basic_tokenizer.zig:6-10 and the std errors the reference propagates)
# ---------------------------------------------------------------------------------------------


class ZbpeError(Exception):
    """Base class for every error this package raises."""


class TrainError(ZbpeError):
    pass


class InvalidVocabSize(TrainError):
    pass


class InvalidUtf8(TrainError):  # declared by the reference, never returned (:8)
    pass


class OutOfMemory(TrainError):
    pass


class DeviceError(ZbpeError):
    """A HIP/RCCL failure. The Zig shim maps this to error.OutOfMemory (TrainError is closed)."""


class InvalidToken(ZbpeError):
    pass


class InvalidFormat(ZbpeError):
    pass


class InvalidCharacter(ZbpeError):
    pass


class Overflow(ZbpeError):
    pass


class StreamTooLong(ZbpeError):
    pass


class InvalidArgument(ZbpeError):
    pass


class InternalError(ZbpeError):
    pass


_STATUS = {
    1: InvalidVocabSize,
    2: OutOfMemory,
    3: DeviceError,
    4: DeviceError,
    5: InvalidArgument,
    6: InvalidToken,
    7: InternalError,
}

# ---------------------------------------------------------------------------------------------
# C ABI (include/zbpe.h)
# ---------------------------------------------------------------------------------------------


class Stats(ctypes.Structure):
    """zbpe_stats: the reference's TimeStats buckets (time_statistics.zig:4-13) + counters."""

    _fields_ = [
        ("count_pairs_s", ctypes.c_double),
        ("sort_pairs_s", ctypes.c_double),
        ("replace_pair_s", ctypes.c_double),
        ("other_s", ctypes.c_double),
        ("total_s", ctypes.c_double),
        ("count_pairs_calls", ctypes.c_uint64),
        ("sort_pairs_calls", ctypes.c_uint64),
        ("replace_pair_calls", ctypes.c_uint64),
        ("scan_launches", ctypes.c_uint64),
        ("scan_kernel_s", ctypes.c_double),
        ("scan_alg_bytes", ctypes.c_uint64),
        ("scan_read_bytes", ctypes.c_uint64),
        ("tie_iterations", ctypes.c_uint64),
        ("tie_fallbacks", ctypes.c_uint64),
        ("compactions", ctypes.c_uint64),
        ("self_pair_merges", ctypes.c_uint64),
        ("final_tokens", ctypes.c_uint64),
        ("distinct_pairs", ctypes.c_uint64),
        ("pair_ids", ctypes.c_uint64),
        ("sum_tokens", ctypes.c_uint64),
        ("scan_timed_launches", ctypes.c_uint64),
        ("scan_timed_alg_bytes", ctypes.c_uint64),
        ("list_scans", ctypes.c_uint64),
        ("list_builds", ctypes.c_uint64),
        ("replications", ctypes.c_uint64),
        ("sharded_s", ctypes.c_double),
        ("replicate_s", ctypes.c_double),
        ("replicated_s", ctypes.c_double),
        ("comm_s", ctypes.c_double),
        ("sharded_merges", ctypes.c_uint64),
        ("tie_crosschecks", ctypes.c_uint64),
        ("generate_tokens_s", ctypes.c_double),
        ("pair_selects", ctypes.c_uint64),
        ("round_merges", ctypes.c_uint64),
    ]

    def as_dict(self) -> dict:
        return {k: getattr(self, k) for k, _ in self._fields_}


EXPORTS = (
    "zbpe_create", "zbpe_comm_unique_id", "zbpe_create_dist", "zbpe_create_dist_host", "zbpe_destroy", "zbpe_last_error",
    "zbpe_train", "zbpe_upload", "zbpe_train_resident", "zbpe_encode", "zbpe_verify_counts", "zbpe_tokens",
    "zbpe_set_option", "zbpe_format_time_stats", "zbpe_bench_scan", "zbpe_bench_train_scan", "zbpe_merge_log", "zbpe_trace", "zbpe_scan_log", "zbpe_compaction_log", "zbpe_halt_log", "zbpe_zig_order_winner", "zbpe_version",
    "zbpe_stats_size", "zbpe_bench_recount",
)
MERGE_LOG_COLUMNS = ("key", "count", "live", "ties", "list_scan", "list_len", "key_live", "range")
TRACE_COLUMNS = ("merge", "count", "live", "slots", "streamed", "scan_ms", "replace_ms", "select_ms", "wall_ms",
                 "self_pair", "ties")

_lib = None
COLLECTIVE_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t)


def torch_collective(rank: int, world: int, group=None):
    """zbpe_collective_fn over torch.distributed (e.g. gloo on the CPU): op 0 sum / op 1 min of u32
    in place, op 2 all-gather of `count` bytes per rank. Used by zbpe_create_dist_host."""
    import torch
    import torch.distributed as dist

    def cb(_user, op, buf, count):
        try:
            if op in (0, 1):
                arr = np.ctypeslib.as_array((ctypes.c_uint32 * count).from_address(buf))
                t = torch.from_numpy(arr.astype(np.int64))
                dist.all_reduce(t, op=dist.ReduceOp.SUM if op == 0 else dist.ReduceOp.MIN, group=group)
                arr[:] = (t.numpy() & 0xFFFFFFFF).astype(np.uint32)
            elif op == 2:
                arr = np.ctypeslib.as_array((ctypes.c_uint8 * (count * world)).from_address(buf))
                mine = torch.from_numpy(arr[rank * count:(rank + 1) * count].copy())
                outs = [torch.empty_like(mine) for _ in range(world)]
                dist.all_gather(outs, mine, group=group)
                arr[:] = torch.cat(outs).numpy()
            else:
                return 2
            return 0
        except Exception as e:  # noqa: BLE001 -- reported to the C side as a failed collective
            sys.stderr.write(f"zbpe collective op {op} failed: {e}\n")
            return 1

    return COLLECTIVE_FN(cb)


def load_library(path: str = LIB_PATH) -> ctypes.CDLL:
    """Load libzbpe.so (built by `make -C zig-bpe_amd` / __graft_entry__.build()). Raises if absent."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise ImportError(f"libzbpe.so not built: {path} (run `make -C zig-bpe_amd` or __graft_entry__.build())")
    L = ctypes.CDLL(path)
    vp, sz, u16p, u64p = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_void_p
    L.zbpe_create.argtypes = [ctypes.c_int, ctypes.POINTER(vp)]
    L.zbpe_comm_unique_id.argtypes = [vp]
    L.zbpe_create_dist.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, vp, ctypes.POINTER(vp)]
    L.zbpe_create_dist_host.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, COLLECTIVE_FN, vp, ctypes.POINTER(vp)]
    L.zbpe_destroy.argtypes = [vp]
    L.zbpe_destroy.restype = None
    L.zbpe_last_error.argtypes = [vp]
    L.zbpe_last_error.restype = ctypes.c_char_p
    L.zbpe_train.argtypes = [vp, vp, sz, ctypes.c_uint16, ctypes.c_int, u16p, u64p, ctypes.POINTER(sz), ctypes.POINTER(Stats)]
    L.zbpe_upload.argtypes = [vp, vp, sz]
    L.zbpe_train_resident.argtypes = [vp, ctypes.c_uint16, ctypes.c_int, u16p, u64p, ctypes.POINTER(sz), ctypes.POINTER(Stats)]
    L.zbpe_encode.argtypes = [vp, u16p, sz, vp, sz, u16p, ctypes.POINTER(sz)]
    L.zbpe_verify_counts.argtypes = [vp, ctypes.POINTER(ctypes.c_uint64)]
    if hasattr(L, "zbpe_tokens"):  # (absent from older builds loaded for A/B runs through ZBPE_LIB)
        L.zbpe_tokens.argtypes = [vp, u16p, sz, ctypes.POINTER(sz)]
        L.zbpe_format_time_stats.argtypes = [ctypes.POINTER(Stats), ctypes.c_char_p, sz, ctypes.POINTER(sz)]
    if hasattr(L, "zbpe_merge_log"):
        L.zbpe_merge_log.argtypes = [vp, vp, sz, ctypes.POINTER(sz)]
    if hasattr(L, "zbpe_bench_train_scan"):
        L.zbpe_bench_train_scan.argtypes = [vp, ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_double),
                                            ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(ctypes.c_uint32),
                                            ctypes.POINTER(ctypes.c_int)]
    if hasattr(L, "zbpe_bench_recount"):
        L.zbpe_bench_recount.argtypes = [vp, ctypes.c_int, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double),
                                         ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64)]
    L.zbpe_set_option.argtypes = [vp, ctypes.c_char_p, ctypes.c_int64]
    L.zbpe_bench_scan.argtypes = [vp, ctypes.c_uint16, ctypes.c_uint16, ctypes.c_int, ctypes.POINTER(ctypes.c_double),
                                  ctypes.POINTER(ctypes.c_double)]
    L.zbpe_trace.argtypes = [vp, vp, sz, ctypes.POINTER(sz)]
    L.zbpe_scan_log.argtypes = [vp, vp, sz, ctypes.POINTER(sz)]
    L.zbpe_compaction_log.argtypes = [vp, vp, sz, ctypes.POINTER(sz)]
    L.zbpe_halt_log.argtypes = [vp, vp, sz, ctypes.POINTER(sz)]
    L.zbpe_zig_order_winner.argtypes = [vp, vp, vp, sz, ctypes.c_uint32, ctypes.c_int, ctypes.POINTER(ctypes.c_uint32)]
    L.zbpe_version.restype = ctypes.c_char_p
    for name in EXPORTS:
        if name not in ("zbpe_destroy", "zbpe_last_error", "zbpe_version", "zbpe_stats_size") and hasattr(L, name):
            getattr(L, name).restype = ctypes.c_int
    if hasattr(L, "zbpe_stats_size"):  # the caller-allocated zbpe_stats must match the library's layout
        L.zbpe_stats_size.restype = ctypes.c_size_t
        if L.zbpe_stats_size() != ctypes.sizeof(Stats):
            raise ImportError(f"{path}: zbpe_stats is {L.zbpe_stats_size()} B, this binding's is {ctypes.sizeof(Stats)} B")
    _lib = L
    return L


def _ptr(a: np.ndarray):
    return a.ctypes.data_as(ctypes.c_void_p)


class Engine:
    """One device context (one GPU). Thin wrapper over the C ABI; not re-entrant (like the reference)."""

    def __init__(self, device: int = 0, rank: int = 0, world: int = 1, unique_id: Optional[bytes] = None,
                 collective=None):
        """world > 1: RCCL with `unique_id` (from comm_unique_id() on rank 0), or a host `collective`
        (torch_collective(rank, world)) so several ranks can share one GPU. world == 1 with a unique_id or a
        collective: a one-rank communicator that runs the sharded code path (tests)."""
        self._L = load_library()
        self._ctx = ctypes.c_void_p()
        self._collective = collective  # keep the callback alive
        if world == 1 and collective is None and unique_id is None:
            st = self._L.zbpe_create(device, ctypes.byref(self._ctx))
        elif collective is not None:
            st = self._L.zbpe_create_dist_host(device, rank, world, collective, None, ctypes.byref(self._ctx))
        else:
            uid = ctypes.create_string_buffer(unique_id or b"", 128)
            st = self._L.zbpe_create_dist(device, rank, world, uid, ctypes.byref(self._ctx))
        if st != 0:
            msg = self._L.zbpe_last_error(self._ctx).decode() if self._ctx else ""
            self.close()
            raise _STATUS.get(st, ZbpeError)(f"zbpe_create failed ({st}): {msg}")
        self.rank, self.world = rank, world

    def _check(self, st: int, what: str):
        if st != 0:
            raise _STATUS.get(st, ZbpeError)(f"{what}: {self._L.zbpe_last_error(self._ctx).decode()}")

    def close(self):
        if getattr(self, "_ctx", None):
            self._L.zbpe_destroy(self._ctx)
            self._ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_option(self, name: str, value: int):
        self._check(self._L.zbpe_set_option(self._ctx, name.encode(), int(value)), f"set_option({name})")

    def upload(self, text: bytes):
        buf = np.frombuffer(text, dtype=np.uint8) if len(text) else np.zeros(1, np.uint8)
        self._check(self._L.zbpe_upload(self._ctx, _ptr(buf), len(text)), "zbpe_upload")

    def _train_out(self, vocab_size: int):
        m = max(vocab_size - vocabStart, 0)
        return np.zeros(3 * max(m, 1), np.uint16), np.zeros(max(m, 1), np.uint64), ctypes.c_size_t(0), Stats()

    def train(self, text: bytes, vocab_size: int, verbose: bool = False):
        """-> (merges (M,3) uint16, counts (M,) uint64, Stats)"""
        if vocab_size < vocabStart:
            raise InvalidVocabSize(f"vocabSize {vocab_size} < 256")
        tri, cnt, nm, st = self._train_out(vocab_size)
        buf = np.frombuffer(text, dtype=np.uint8) if len(text) else np.zeros(1, np.uint8)
        self._check(self._L.zbpe_train(self._ctx, _ptr(buf), len(text), vocab_size, int(verbose), _ptr(tri), _ptr(cnt),
                                       ctypes.byref(nm), ctypes.byref(st)), "zbpe_train")
        m = nm.value
        return tri[: 3 * m].reshape(m, 3).copy(), cnt[:m].copy(), st

    def train_resident(self, vocab_size: int, verbose: bool = False):
        if vocab_size < vocabStart:
            raise InvalidVocabSize(f"vocabSize {vocab_size} < 256")
        tri, cnt, nm, st = self._train_out(vocab_size)
        self._check(self._L.zbpe_train_resident(self._ctx, vocab_size, int(verbose), _ptr(tri), _ptr(cnt),
                                                ctypes.byref(nm), ctypes.byref(st)), "zbpe_train_resident")
        m = nm.value
        return tri[: 3 * m].reshape(m, 3).copy(), cnt[:m].copy(), st

    def encode(self, merges: np.ndarray, text: bytes) -> np.ndarray:
        tri = np.ascontiguousarray(np.asarray(merges, dtype=np.uint16).reshape(-1))
        tri_p = tri if len(tri) else np.zeros(3, np.uint16)
        out = np.zeros(max(len(text), 1), np.uint16)
        n = ctypes.c_size_t(0)
        buf = np.frombuffer(text, dtype=np.uint8) if len(text) else np.zeros(1, np.uint8)
        self._check(self._L.zbpe_encode(self._ctx, _ptr(tri_p), len(tri) // 3, _ptr(buf), len(text), _ptr(out),
                                        ctypes.byref(n)), "zbpe_encode")
        return out[: n.value].copy()

    def bench_scan(self, a: int, b: int, reps: int = 10):
        ms, gbps = ctypes.c_double(0), ctypes.c_double(0)
        self._check(self._L.zbpe_bench_scan(self._ctx, a, b, reps, ctypes.byref(ms), ctypes.byref(gbps)), "zbpe_bench_scan")
        return ms.value, gbps.value

    def bench_train_scan(self, reps: int = 20, grid: int = 0) -> dict:
        """Late-phase scan microbenchmark on the trained state (zbpe_bench_train_scan)."""
        us, pair, ln, mode = ctypes.c_double(0), ctypes.c_uint32(0), ctypes.c_uint32(0), ctypes.c_int(0)
        self._check(self._L.zbpe_bench_train_scan(self._ctx, reps, grid, ctypes.byref(us), ctypes.byref(pair), ctypes.byref(ln),
                                                  ctypes.byref(mode)), "zbpe_bench_train_scan")
        return {"us": us.value, "pair": (pair.value & 0xFFFF, pair.value >> 16), "list_len": ln.value, "mode": mode.value}

    def bench_recount(self, reps: int = 5) -> dict:
        """Full pair-histogram kernel timing on the trained state (zbpe_bench_recount)."""
        us, gbps, n, mm = ctypes.c_double(0), ctypes.c_double(0), ctypes.c_uint64(0), ctypes.c_uint64(0)
        self._check(self._L.zbpe_bench_recount(self._ctx, reps, ctypes.byref(us), ctypes.byref(gbps), ctypes.byref(n),
                                               ctypes.byref(mm)), "zbpe_bench_recount")
        return {"us": us.value, "GBps": gbps.value, "tokens": n.value, "mismatches": mm.value}

    def trace(self):
        """Per-merge rows of the last train (option "trace" = 1): float32 array [merges, len(TRACE_COLUMNS)]."""
        import numpy as np

        n = ctypes.c_size_t(0)
        self._check(self._L.zbpe_trace(self._ctx, None, 0, ctypes.byref(n)), "zbpe_trace")
        out = np.zeros((n.value, len(TRACE_COLUMNS)), dtype=np.float32)
        if n.value:
            self._check(self._L.zbpe_trace(self._ctx, _ptr(out), n.value, ctypes.byref(n)), "zbpe_trace")
        return out

    def merge_log(self) -> np.ndarray:
        """Device per-merge log of the last train: uint32 [merges, 8] (see MERGE_LOG_COLUMNS)."""
        n = ctypes.c_size_t(0)
        self._check(self._L.zbpe_merge_log(self._ctx, None, 0, ctypes.byref(n)), "zbpe_merge_log")
        out = np.zeros((n.value, 8), dtype=np.uint32)
        if n.value:
            self._check(self._L.zbpe_merge_log(self._ctx, _ptr(out), n.value, ctypes.byref(n)), "zbpe_merge_log")
        return out

    def scan_log(self) -> np.ndarray:
        """Per pair-scan launch of the last train: 2 * merge index + form (0 stream, 1 list), -1 = no-op launch."""
        n = ctypes.c_size_t(0)
        self._check(self._L.zbpe_scan_log(self._ctx, None, 0, ctypes.byref(n)), "zbpe_scan_log")
        out = np.zeros(n.value, dtype=np.int32)
        if n.value:
            self._check(self._L.zbpe_scan_log(self._ctx, _ptr(out), n.value, ctypes.byref(n)), "zbpe_scan_log")
        return out

    def compaction_log(self) -> np.ndarray:
        """Per stream compaction of the last train: (merge token X, replicated arena fill arena_rep)."""
        n = ctypes.c_size_t(0)
        self._check(self._L.zbpe_compaction_log(self._ctx, None, 0, ctypes.byref(n)), "zbpe_compaction_log")
        out = np.zeros((n.value, 2), dtype=np.uint32)
        if n.value:
            self._check(self._L.zbpe_compaction_log(self._ctx, _ptr(out), n.value, ctypes.byref(n)), "zbpe_compaction_log")
        return out

    def halt_log(self) -> np.ndarray:
        """Per halted device-resident batch of the last train: (merge token X, HaltReason, host-path microseconds)."""
        n = ctypes.c_size_t(0)
        self._check(self._L.zbpe_halt_log(self._ctx, None, 0, ctypes.byref(n)), "zbpe_halt_log")
        out = np.zeros((n.value, 3), dtype=np.uint32)
        if n.value:
            self._check(self._L.zbpe_halt_log(self._ctx, _ptr(out), n.value, ctypes.byref(n)), "zbpe_halt_log")
        return out

    def tokens(self) -> np.ndarray:
        """The current token stream (after the last train: expandVocabulary's currentTokens), as uint16."""
        n = ctypes.c_size_t(0)
        self._check(self._L.zbpe_tokens(self._ctx, None, 0, ctypes.byref(n)), "zbpe_tokens")
        out = np.zeros(max(n.value, 1), dtype=np.uint16)
        self._check(self._L.zbpe_tokens(self._ctx, _ptr(out), n.value, ctypes.byref(n)), "zbpe_tokens")
        return out[: n.value]

    def verify_counts(self) -> int:
        mm = ctypes.c_uint64(0)
        self._check(self._L.zbpe_verify_counts(self._ctx, ctypes.byref(mm)), "zbpe_verify_counts")
        return int(mm.value)


def format_time_stats(st: Stats) -> str:
    """printTimeStats (time_statistics.zig:36-60) text for a train's Stats."""
    L = load_library()
    n = ctypes.c_size_t(0)
    buf = ctypes.create_string_buffer(1024)
    if L.zbpe_format_time_stats(ctypes.byref(st), buf, 1024, ctypes.byref(n)) != 0:
        raise InvalidArgument("zbpe_format_time_stats")
    return buf.value.decode()


def comm_unique_id() -> bytes:
    L = load_library()
    buf = ctypes.create_string_buffer(128)
    st = L.zbpe_comm_unique_id(buf)
    if st != 0:
        raise DeviceError(f"zbpe_comm_unique_id failed ({st})")
    return buf.raw


def zig_order_winner(first_pos: Sequence[int], keys: Sequence[int], counts: Sequence[int], top: int,
                     call_after_last_insert: bool) -> int:
    """Host Zig-map emulation used by the engine's exact tie fallback (pure host code, no device)."""
    L = load_library()
    f = np.ascontiguousarray(first_pos, dtype=np.uint32)
    k = np.ascontiguousarray(keys, dtype=np.uint32)
    c = np.ascontiguousarray(counts, dtype=np.uint32)
    w = ctypes.c_uint32(0)
    st = L.zbpe_zig_order_winner(_ptr(f), _ptr(k), _ptr(c), len(f), top, int(call_after_last_insert), ctypes.byref(w))
    if st != 0:
        raise InternalError("no pair with the top count")
    return int(w.value)


# ---------------------------------------------------------------------------------------------
# corpus generator (bench/test harness, zig-bpe_amd/csrc/synth_corpus.c)
# ---------------------------------------------------------------------------------------------
_synth = None

CORPUS_KINDS = {"words": 0, "words_utf8": 1, "uniform": 2, "runs": 3}


def synth_corpus(kind: str, seed: int, n: int, utf8_permille: int = 50, threads: int = 8) -> bytes:
    global _synth
    if _synth is None:
        if not os.path.exists(SYNTH_PATH):
            raise ImportError(f"{SYNTH_PATH} not built")
        _synth = ctypes.CDLL(SYNTH_PATH)
        _synth.zbpe_synth_corpus.argtypes = [ctypes.c_int, ctypes.c_uint64, ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t,
                                             ctypes.c_int]
    buf = np.zeros(max(n, 1), np.uint8)
    rc = _synth.zbpe_synth_corpus(CORPUS_KINDS[kind], seed, utf8_permille, _ptr(buf), n, threads)
    if rc:
        raise ValueError(f"synth_corpus({kind}) failed: {rc}")
    return buf[:n].tobytes()


# ---------------------------------------------------------------------------------------------
# host-side mirror of the reference data model and struct API
# ---------------------------------------------------------------------------------------------


@dataclass(frozen=True)
class CharPair:  # basic_tokenizer.zig:40-43
    first: int
    second: int


@dataclass(frozen=True)
class Merge:  # :12-15
    pair: CharPair
    new_token: int


@dataclass
class Merges:  # :17-38
    merges: List[Merge] = field(default_factory=list)

    def put(self, pair: CharPair, new_token: int) -> None:
        self.merges.append(Merge(pair, int(new_token)))

    def as_array(self) -> np.ndarray:
        return np.array([[m.pair.first, m.pair.second, m.new_token] for m in self.merges], dtype=np.uint16).reshape(-1, 3)


def _parse_u16(s: bytes) -> int:
    """std.fmt.parseInt(u16, s, 10) (Zig 0.13): optional sign, digits, '_' only between digits."""
    if len(s) == 0:
        raise InvalidCharacter("empty field")
    neg = False
    if s[:1] in (b"+", b"-"):
        neg = s[:1] == b"-"
        s = s[1:]
    if len(s) == 0 or s[:1] == b"_" or s[-1:] == b"_":
        raise InvalidCharacter(repr(s))
    v = 0
    for ch in s:
        if ch == ord("_"):
            continue
        if not (48 <= ch <= 57):
            raise InvalidCharacter(repr(s))
        v = v * 10 + (ch - 48)
        if v > 0xFFFF and not neg:
            raise Overflow(repr(s))
    if neg:
        if v != 0:
            raise Overflow(repr(s))
        return 0
    return v


class BasicTokenizer:
    """Drop-in mirror of the reference struct (basic_tokenizer.zig:52-349)."""

    def __init__(self, device: int = 0, engine: Optional[Engine] = None):
        self.merges = Merges()
        # TimeStats.init (time_statistics.zig:15-29): created once, accumulated over every train call
        self.timeStats: Stats = Stats()
        self._device = device
        self._engine = engine

    # init / deinit (:57-69)
    @classmethod
    def init(cls, device: int = 0) -> "BasicTokenizer":
        return cls(device)

    def deinit(self) -> None:
        if self._engine is not None:
            self._engine.close()
            self._engine = None
        self.merges = Merges()

    @property
    def engine(self) -> Engine:
        if self._engine is None:
            self._engine = Engine(self._device)
        return self._engine

    # train (:140-153): appends to merges (the reference never clears them, :199)
    def train(self, text: bytes, vocabSize: int, verbose: bool = False) -> None:
        # the reference prints printTimeStats from a defer (:141-145): on every way out, errors included,
        # with the accumulated buckets and this call's own total time
        start = time.perf_counter()
        try:
            if isinstance(text, str):
                text = text.encode()
            if vocabSize < vocabStart:
                raise InvalidVocabSize(f"vocabSize {vocabSize} < 256")
            if vocabSize > 0xFFFF:
                raise InvalidArgument("vocabSize is a u16")
            tri, _counts, st = self.engine.train(text, vocabSize, verbose)
            for a, b, x in tri:
                self.merges.put(CharPair(int(a), int(b)), int(x))
            acc = self.timeStats
            for k in ("count_pairs_s", "sort_pairs_s", "replace_pair_s", "other_s", "total_s", "count_pairs_calls",
                      "sort_pairs_calls", "replace_pair_calls", "generate_tokens_s"):
                setattr(acc, k, getattr(acc, k) + getattr(st, k))
        finally:
            shown = Stats.from_buffer_copy(self.timeStats)
            shown.total_s = time.perf_counter() - start
            sys.stderr.write(format_time_stats(shown))

    # encode (:71-88)
    def encode(self, text: bytes) -> List[int]:
        if isinstance(text, str):
            text = text.encode()
        return self.engine.encode(self.merges.as_array(), text).tolist()

    # decode (:90-138): first merge with that new_token, recursive left then right
    def _find_merge(self, token: int) -> Optional[Merge]:
        for m in self.merges.merges:
            if m.new_token == token:
                return m
        return None

    def decode(self, tokens: Iterable[int]) -> bytes:
        by_token = {}
        for m in self.merges.merges:  # first match wins (findMerge :109-116)
            by_token.setdefault(m.new_token, m)
        out = bytearray()
        sys.setrecursionlimit(max(sys.getrecursionlimit(), 100000))

        def expand(m: Merge, depth: int = 0):
            if depth > 70000:
                raise InvalidToken("merge cycle")
            for t in (m.pair.first, m.pair.second):
                if t < 256:
                    out.append(t)
                else:
                    sub = by_token.get(t)
                    if sub is None:
                        raise InvalidToken(str(t))
                    expand(sub, depth + 1)

        for t in tokens:
            t = int(t)
            if t < 256:
                out.append(t)
            else:
                m = by_token.get(t)
                if m is None:
                    raise InvalidToken(str(t))
                expand(m)
        return bytes(out)

    # serializeMerges (:319-330)
    def serializeMerges(self, file_path: str) -> None:
        with open(file_path, "wb") as f:
            for m in self.merges.merges:
                f.write(f"{m.pair.first},{m.pair.second},{m.new_token}\n".encode())

    # deserializeMerges (:332-348): 100-byte line buffer, split on ',', three u16 fields, appends
    def deserializeMerges(self, file_path: str) -> None:
        with open(file_path, "rb") as f:
            data = f.read()
        pos = 0
        while pos < len(data):
            nl = data.find(b"\n", pos, pos + 100)
            if nl < 0:
                if len(data) - pos >= 100:
                    raise StreamTooLong(f"line at byte {pos}")
                line, pos = data[pos:], len(data)
            else:
                line, pos = data[pos:nl], nl + 1
            fields = line.split(b",")
            if len(fields) < 1:
                raise InvalidFormat(repr(line))
            first = _parse_u16(fields[0])
            if len(fields) < 2:
                raise InvalidFormat(repr(line))
            second = _parse_u16(fields[1])
            if len(fields) < 3:
                raise InvalidFormat(repr(line))
            new_token = _parse_u16(fields[2])
            self.merges.put(CharPair(first, second), new_token)


def merges_to_text(merges: np.ndarray) -> bytes:
    return "".join(f"{int(a)},{int(b)},{int(c)}\n" for a, b, c in np.asarray(merges).reshape(-1, 3)).encode()


__all__ = [
    "BasicTokenizer", "CharPair", "Merge", "Merges", "Engine", "Stats", "TrainError", "InvalidVocabSize", "InvalidUtf8",
    "OutOfMemory", "DeviceError", "InvalidToken", "InvalidFormat", "InvalidCharacter", "Overflow", "StreamTooLong",
    "InvalidArgument", "InternalError", "load_library", "synth_corpus", "comm_unique_id", "zig_order_winner",
    "merges_to_text", "format_time_stats", "vocabStart", "EXPORTS", "TRACE_COLUMNS", "torch_collective", "COLLECTIVE_FN",
]
