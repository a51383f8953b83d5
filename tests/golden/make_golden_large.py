"""Full-sequence oracle goldens at BASELINE.json scale (test infrastructure; run in the dev container).

The oracle (oracle/zig_ref.c, the literal restatement of basic_tokenizer.zig:140-306 with the Zig 0.13
map / Wyhash / stable sort) runs the reference loop unconditionally from the raw bytes:

  c3   configs[2]: words_utf8, seed 0x5EED0003, 64 MiB, vocab 4096 -> all 3,840 merges
  c4   configs[3]: words_utf8, seed 0x5EED0004, 1 GiB, vocab 32000 -> the first K merges (a prefix;
       one literal iteration over the 1 GiB stream takes ~3 s on one core, the full run ~days)

Each run streams one line per merge into a progress log (zref_train_log), so a run that is stopped
keeps its prefix; `convert` turns a (possibly partial) log into the committed JSON:

  python tests/golden/make_golden_large.py run c3 /tmp/zbpe_golden/c3.log
  python tests/golden/make_golden_large.py run c4 /tmp/zbpe_golden/c4.log [max_merges]
  python tests/golden/make_golden_large.py convert c3 /tmp/zbpe_golden/c3.log

The second oracle (oracle/zig_fast.cpp) runs C4 to the end in a few hours on 8 cores and gives the full golden
(large_c4_words_utf8_1GiB_v32000.json, every tie confirmed by a literal map replay):

  python tests/golden/make_golden_large.py run-fast c4 /tmp/zbpe_golden/c4fast.log [threads]
  python tests/golden/make_golden_large.py convert-fast c4 /tmp/zbpe_golden/c4fast.log

The JSON holds, per merge k: the triple, the top count, the number of pairs tied at it, the distinct
pairs D_k and the stream length after the merge, plus FNV-1a-64 checksums of the stream every
`FNV_EVERY` merges (tests/test_gpu_large.py compares the device's run with all of it).
"""
import ctypes
import hashlib
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "zig-bpe_amd"))
import numpy as np  # noqa: E402

RUNS = {
    # name: (kind, seed, n_bytes, vocab, golden file)
    "c3": ("words_utf8", 0x5EED0003, 64 << 20, 4096, "large_c3_words_utf8_64MiB_v4096.json"),
    "c4": ("words_utf8", 0x5EED0004, 1 << 30, 32000, "large_c4_words_utf8_1GiB_v32000_prefix.json"),
}
FNV_EVERY = 64


def run(name: str, log: str, max_merges: int = 0) -> None:
    import oracle as O
    import zbpe
    kind, seed, n, vocab, _ = RUNS[name]
    text = zbpe.synth_corpus(kind, seed, n, threads=8)
    print(name, "corpus sha256", hashlib.sha256(text).hexdigest(), flush=True)
    L = O.lib()
    cap = vocab - 256
    tri = np.zeros(3 * cap, np.uint16)
    cnt = np.zeros(cap, np.uint64)
    ties = np.zeros(cap, np.uint32)
    dist = np.zeros(cap, np.uint32)
    nm, nt = ctypes.c_size_t(0), ctypes.c_size_t(0)
    st = O.ZrefStats()
    buf = np.frombuffer(text, np.uint8)
    os.makedirs(os.path.dirname(os.path.abspath(log)), exist_ok=True)
    rc = L.zref_train_log(O._p(buf), ctypes.c_size_t(n), ctypes.c_uint32(vocab), ctypes.c_int(0),
                          ctypes.c_uint32(max_merges), O._p(tri), O._p(cnt), O._p(ties), O._p(dist),
                          ctypes.byref(nm), ctypes.byref(st), None, ctypes.byref(nt),
                          os.path.abspath(log).encode(), ctypes.c_uint32(FNV_EVERY))
    print(name, "rc", rc, "merges", nm.value, "final tokens", nt.value, "seconds", round(st.total_s, 1), flush=True)


def run_fast(name: str, log: str, threads: int = 7) -> None:
    """The second oracle (oracle/zig_fast.cpp: incremental counts, a literal Zig-map replay at every
    tied merge) over the whole run; C4 in a few hours on 8 cores."""
    import oracle as O
    import zbpe
    kind, seed, n, vocab, _ = RUNS[name]
    text = zbpe.synth_corpus(kind, seed, n, threads=8)
    print(name, "corpus sha256", hashlib.sha256(text).hexdigest(), flush=True)
    os.makedirs(os.path.dirname(os.path.abspath(log)), exist_ok=True)
    r = O.fast_train(text, vocab, threads=threads, fnv_every=FNV_EVERY, progress=os.path.abspath(log))
    print(name, "merges", len(r.merges), "final tokens", len(r.tokens), "restarts", r.restarts,
          "ties replayed before the merge", r.ties_sync, "ties replayed by workers", r.ties_async, flush=True)


def convert(name: str, log: str) -> str:
    kind, seed, n, vocab, fname = RUNS[name]
    merges, counts, ties, distinct, lens, fnv, done = [], [], [], [], [], [], None
    with open(log) as f:
        for line in f:
            p = line.split()
            if not p:
                continue
            if p[0] == "fnv":
                fnv.append([int(p[1]), int(p[2]), p[3]])
            elif p[0] == "done":
                done = [int(p[1]), int(p[2]), p[3]]
            elif len(p) == 8:
                k = int(p[0])
                assert k == len(merges), (k, len(merges))
                merges.append([int(p[1]), int(p[2]), int(p[3])])
                counts.append(int(p[4]))
                ties.append(int(p[5]))
                distinct.append(int(p[6]))
                lens.append(int(p[7]))
    import zbpe
    corpus_sha = hashlib.sha256(zbpe.synth_corpus(kind, seed, n, threads=8)).hexdigest()
    complete = done is not None and done[0] == vocab - 256
    if done is not None and done[0] == len(merges):
        fnv = [x for x in fnv if x[0] != done[0]] + [done]
    out = {
        "source": "oracle/zig_ref.c zref_train_log (literal restatement of basic_tokenizer.zig:140-306), "
                  "tests/golden/make_golden_large.py",
        "kind": kind, "seed": seed, "n": n, "vocab_size": vocab, "corpus_sha256": corpus_sha,
        "complete": complete, "n_merges": len(merges),
        "merges": merges, "counts": counts, "ties": ties, "distinct": distinct, "len_after": lens,
        "fnv64_after": fnv,
    }
    path = os.path.join(HERE, fname)
    with open(path, "w") as f:
        json.dump(out, f, separators=(",", ":"))
        f.write("\n")
    print(path, len(merges), "merges", sum(t > 1 for t in ties), "tied", "complete" if complete else "prefix")
    return path


def convert_fast(name: str, log: str) -> str:
    """The fast oracle's progress log -> the full-sequence golden (large_<...>.json without `_prefix`). A run
    that restarted (a replay overruled a predicted tie winner) logs `restart`; only the last attempt counts.
    `complete` needs the final `done` line and a confirming replay for every tied merge."""
    kind, seed, n, vocab, fname = RUNS[name]
    # C4: the full golden beside the literal oracle's prefix; other runs keep the literal oracle's file
    fname = fname.replace("_prefix", "") if "_prefix" in fname else fname.replace(".json", "_fast.json")
    merges, counts, ties, distinct, lens, fnv, done = [], [], [], [], [], {}, None
    ok, bad, restarts, sync, timing = set(), 0, 0, 0, None
    with open(log) as f:
        for line in f:
            p = line.split()
            if not p:
                continue
            if p[0] == "restart":
                restarts += 1
                merges, counts, ties, distinct, lens, fnv, ok, bad, sync = [], [], [], [], [], {}, set(), 0, 0
            elif p[0] == "fnv":
                fnv[int(p[1])] = [int(p[1]), int(p[2]), p[3]]
            elif p[0] == "done":
                done = [int(p[1]), int(p[2]), p[3]]
            elif p[0] == "tie":
                if p[2] == "ok":
                    ok.add(int(p[1]))
                    sync += p[-1] == "sync"
                else:
                    bad += 1
            elif p[0] == "timing":
                timing = {p[i]: float(p[i + 1]) for i in range(1, len(p) - 1, 2)}
            elif len(p) == 8 and p[0].isdigit():
                k = int(p[0])
                assert k == len(merges), (k, len(merges))
                merges.append([int(p[1]), int(p[2]), int(p[3])])
                counts.append(int(p[4]))
                ties.append(int(p[5]))
                distinct.append(int(p[6]))
                lens.append(int(p[7]))
    tied = [k for k, t in enumerate(ties) if t > 1]
    confirmed = all(k in ok for k in tied)
    import zbpe
    corpus_sha = hashlib.sha256(zbpe.synth_corpus(kind, seed, n, threads=8)).hexdigest()
    complete = done is not None and done[0] == vocab - 256 == len(merges) and confirmed and bad == 0
    if done is not None and done[0] == len(merges):
        fnv[done[0]] = done
    out = {
        "source": "oracle/zig_fast.cpp zfast_train (incremental restatement of basic_tokenizer.zig:140-306: exact "
                  "incremental counts, a literal Zig 0.13 HashMapUnmanaged replay in first-occurrence order at every "
                  "tied merge), tests/golden/make_golden_large.py run-fast / convert-fast",
        "kind": kind, "seed": seed, "n": n, "vocab_size": vocab, "corpus_sha256": corpus_sha,
        "complete": complete, "n_merges": len(merges),
        "merges": merges, "counts": counts, "ties": ties, "distinct": distinct, "len_after": lens,
        "fnv64_after": [fnv[k] for k in sorted(fnv)],
        "tie_replays": {"replayed": len(ok & set(tied)), "before_the_merge": sync, "mismatches": bad,
                        "restarts": restarts},
        "oracle_timing_s": timing,
    }
    path = os.path.join(HERE, fname)
    with open(path, "w") as f:
        json.dump(out, f, separators=(",", ":"))
        f.write("\n")
    print(path, len(merges), "merges", len(tied), "tied", len(ok), "replays confirmed", bad, "mismatches",
          "complete" if complete else "INCOMPLETE")
    return path


if __name__ == "__main__":
    cmd, name, log = sys.argv[1], sys.argv[2], sys.argv[3]
    if cmd == "run":
        run(name, log, int(sys.argv[4]) if len(sys.argv) > 4 else 0)
    elif cmd == "run-fast":
        run_fast(name, log, int(sys.argv[4]) if len(sys.argv) > 4 else 7)
    elif cmd == "convert":
        convert(name, log)
    elif cmd == "convert-fast":
        convert_fast(name, log)
    else:
        raise SystemExit(f"unknown command {cmd}")
