"""Regenerates the committed golden fixtures (run in the dev container; needs /root/reference
for the C1 files). Test infrastructure: uses the CPU oracle (oracle/zig_ref.c).

  c1_taylorswift.txt.gz  reference data file /root/reference/taylorswift.txt (gzip, byte-identical)
  c1_merges.json         reference output /root/reference/merges.txt as triples + the oracle's
                         per-merge counts/ties/distinct pairs (counts are oracle-derived: the
                         reference ships only the merges)
  synth_*.json           oracle outputs on seeded synthetic corpora (regenerated on the GPU box by
                         zbpe.synth_corpus from kind/seed/n)
"""
import gzip
import hashlib
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "zig-bpe_amd"))
import numpy as np  # noqa: E402
import oracle as O  # noqa: E402
import zbpe  # noqa: E402

SYNTH = [
    # name, kind, seed, n, vocab
    ("c2_words_1MiB_v512", "words", 0x5EED0002, 1 << 20, 512),
    ("utf8_256KiB_v600", "words_utf8", 3, 1 << 18, 600),
    ("uniform_64KiB_v400", "uniform", 7, 1 << 16, 400),
    ("runs_64KiB_v320", "runs", 9, 1 << 16, 320),
    ("uniform_4KiB_exhaust", "uniform", 11, 4096, 1000),
    ("runs_3000_exhaust", "runs", 12, 3000, 600),
    ("words_20000_v2000", "words", 13, 20000, 2000),
]


def dump(path, obj):
    with open(path, "w") as f:
        json.dump(obj, f, separators=(",", ":"))
        f.write("\n")


def main():
    ref = "/root/reference"
    if os.path.isdir(ref):
        text = open(os.path.join(ref, "taylorswift.txt"), "rb").read()
        merges_txt = open(os.path.join(ref, "merges.txt"), "rb").read()
        with gzip.GzipFile(os.path.join(HERE, "c1_taylorswift.txt.gz"), "wb", mtime=0) as g:
            g.write(text)
        r = O.train(text, 300)
        assert O.serialize(r.merges) == merges_txt, "oracle does not reproduce merges.txt"
        triples = [[int(a), int(b), int(c)] for a, b, c in (l.split(b",") for l in merges_txt.splitlines())]
        dump(os.path.join(HERE, "c1_merges.json"), {
            "source": "reference merges.txt (main.zig:21-22: train(taylorswift.txt, 300))",
            "taylorswift_sha256": hashlib.sha256(text).hexdigest(),
            "merges_txt_sha256": hashlib.sha256(merges_txt).hexdigest(),
            "vocab_size": 300, "merges": triples,
            "oracle_counts": [int(c) for c in r.counts], "oracle_ties": [int(t) for t in r.ties],
            "oracle_distinct": [int(d) for d in r.distinct], "oracle_final_tokens": int(len(r.tokens)),
        })
    for name, kind, seed, n, vocab in SYNTH:
        text = zbpe.synth_corpus(kind, seed, n)
        r = O.train(text, vocab)
        dump(os.path.join(HERE, f"synth_{name}.json"), {
            "kind": kind, "seed": seed, "n": n, "vocab_size": vocab,
            "corpus_sha256": hashlib.sha256(text).hexdigest(),
            "merges": r.merges.astype(int).tolist(), "counts": [int(c) for c in r.counts],
            "ties": [int(t) for t in r.ties], "distinct": [int(d) for d in r.distinct],
            "final_tokens": int(len(r.tokens)), "final_tokens_sha256": hashlib.sha256(r.tokens.tobytes()).hexdigest(),
        })
        print(name, len(r.merges), "merges", int((r.ties > 1).sum()), "tie iterations")


if __name__ == "__main__":
    main()
