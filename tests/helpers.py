"""Shared test helpers: golden fixtures (tests/golden) and corpus regeneration."""
import glob
import gzip
import hashlib
import json
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def c1_text() -> bytes:
    with gzip.open(os.path.join(GOLDEN, "c1_taylorswift.txt.gz"), "rb") as f:
        return f.read()


def c1_golden() -> dict:
    with open(os.path.join(GOLDEN, "c1_merges.json")) as f:
        return json.load(f)


def c1_merges_txt() -> bytes:
    return "".join(f"{a},{b},{c}\n" for a, b, c in c1_golden()["merges"]).encode()


def synth_goldens():
    out = []
    for p in sorted(glob.glob(os.path.join(GOLDEN, "synth_*.json"))):
        with open(p) as f:
            g = json.load(f)
        g["name"] = os.path.basename(p)[6:-5]
        out.append(g)
    return out


def synth_text(g: dict) -> bytes:
    import zbpe

    t = zbpe.synth_corpus(g["kind"], g["seed"], g["n"])
    assert hashlib.sha256(t).hexdigest() == g["corpus_sha256"], "corpus generator changed"
    return t


def sha256(b) -> str:
    return hashlib.sha256(bytes(b)).hexdigest()


def as_triples(m) -> np.ndarray:
    return np.asarray(m, dtype=np.uint16).reshape(-1, 3)
