"""Loaders for the golden vectors captured from the real reference libbine.

The fixtures (tests/golden/index.json.gz + outputs.npz) were produced by
tools/make_golden.py from oracle/_ref (the reference's own libbine sources
compiled against MPICH 3.3.2); see that script for the case matrix.  Stored
outputs are kept once per distinct content: a stored case names its npz
member in "blob".
"""
from __future__ import annotations

import functools
import gzip
import hashlib
import json
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
from oracle.oracle import NP_DTYPES as NP  # noqa: E402  (pair types: structured dtypes)


@functools.lru_cache(maxsize=None)
def cases():
    with gzip.open(os.path.join(GOLDEN, "index.json.gz"), "rt") as f:
        return json.load(f)["cases"]


@functools.lru_cache(maxsize=None)
def _npz():
    return np.load(os.path.join(GOLDEN, "outputs.npz"), allow_pickle=False)


def select(**kw):
    out = []
    for c in cases():
        if all(c.get(k) == v for k, v in kw.items()):
            out.append(c)
    return out


def rcounts(c):
    P, N = c["P"], c["N"]
    return [N // P + ((i % 3) if c["rcounts"].startswith("ragged") else 0) for i in range(P)]


def root(c):
    """bcast cases: rcounts "root<k>" = root k, else 0 (oracle/ref_golden.c)"""
    return int(c["rcounts"][4:]) if c["rcounts"].startswith("root") else 0


def inputs(c, total=None):
    """every rank's send buffer of case c (pico_core's generator, seed_base +
    rank; sparsified for the "*_sparse" input kinds, oracle/ref_golden.c)"""
    from oracle import oracle as O
    n = c["N"] if total is None else total
    return O.inputs(c["dtype"], n, c["P"], c["seed_base"], sparse=c["rcounts"].endswith("_sparse"))


def sha(a: np.ndarray) -> str:
    from oracle.oracle import canonical   # pair types: padding zeroed, as in the fixtures
    return hashlib.sha256(canonical(np.asarray(a))).hexdigest()


def outputs(c):
    """Per-rank expected outputs of a stored case (list of arrays), else None."""
    if not c.get("stored"):
        return None
    raw = _npz()[c["blob"]].tobytes()
    dt = NP[c["dtype"]]
    if c["stored"] == "rank0":
        a = np.frombuffer(raw, dtype=dt)
        return [a] * c["P"]
    res, off = [], 0
    esz = np.dtype(dt).itemsize
    for n in c["outn"]:
        res.append(np.frombuffer(raw[off:off + n * esz], dtype=dt))
        off += n * esz
    return res


def check_rank_outputs(c, got, ranks=None):
    """Assert that per-rank outputs `got` equal the golden bit-for-bit
    (digest comparison; identical to a byte compare)."""
    ranks = range(c["P"]) if ranks is None else ranks
    bad = [r for r in ranks if sha(np.asarray(got[r])[: c["outn"][r]]) != c["sha256"][r]]
    return bad
