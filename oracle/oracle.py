"""ctypes front-end of the CPU restatement (oracle/bine_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, by ``__graft_entry__.smoke()`` as
the checker, and by bench.py's ``cpu_baseline`` leg.  The product package
(pico_amd) never imports this module.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = os.path.join(_HERE, "liboracle.so")

DTYPES = {"int8": 0, "uint8": 1, "int16": 2, "uint16": 3, "int32": 4, "uint32": 5,
          "int64": 6, "uint64": 7, "float": 8, "double": 9,
          "float_int": 10, "double_int": 11, "long_int": 12, "2int": 13, "short_int": 14,
          "c_float_complex": 15, "c_double_complex": 16}


def _pair(v: str, size: int) -> np.dtype:
    """C layout of MPI's {value; int index} pair types (index after the value,
    aligned to 4 B; the struct padded to the value's alignment)"""
    off = 4 if v == "<i2" else np.dtype(v).itemsize
    return np.dtype({"names": ["v", "i"], "formats": [v, "<i4"], "offsets": [0, off], "itemsize": size})


NP_DTYPES = {"int8": np.int8, "uint8": np.uint8, "int16": np.int16, "uint16": np.uint16,
             "int32": np.int32, "uint32": np.uint32, "int64": np.int64, "uint64": np.uint64,
             "float": np.float32, "double": np.float64,
             "float_int": _pair("<f4", 8), "double_int": _pair("<f8", 16), "long_int": _pair("<i8", 16),
             "2int": _pair("<i4", 8), "short_int": _pair("<i2", 8),
             "c_float_complex": np.complex64, "c_double_complex": np.complex128}
PAIRS = ("float_int", "double_int", "long_int", "2int", "short_int")
OPS = {"sum": 0, "prod": 1, "max": 2, "min": 3, "land": 4, "band": 5, "lor": 6, "bor": 7, "lxor": 8, "bxor": 9,
       "maxloc": 10, "minloc": 11}


def canonical(a: np.ndarray) -> bytes:
    """the bytes of `a` with the padding of MPI's pair types zeroed: padding is
    not part of the type map (MPICH moves only the fields between ranks, the
    golden harness zeroes it in the reference's outputs), and numpy itself
    does not carry it through copies of padded structured arrays"""
    a = np.ascontiguousarray(a)
    if a.dtype.names:
        z = np.zeros(a.shape, a.dtype)
        for f in a.dtype.names:
            z[f] = a[f]
        return z.tobytes()
    return a.tobytes()
OK, ERR_ARG, ERR_SIZE, ASSERT, DEADLOCK = 0, 12, 51, -2, -3

_lib = None


def build() -> str:
    """Compile liboracle.so (gcc) if missing or stale."""
    src = os.path.join(_HERE, "bine_oracle.c")
    if (not os.path.exists(_LIB)) or os.path.getmtime(_LIB) < os.path.getmtime(src):
        subprocess.run(["make", "-s", "-C", _HERE, "liboracle.so"], check=True)
    return _LIB


def lib():
    global _lib
    if _lib is None:
        build()
        L = ctypes.CDLL(_LIB)
        vp, sz = ctypes.c_void_p, ctypes.c_size_t
        L.orc_fill.argtypes = [vp, ctypes.c_int, sz, ctypes.c_uint]
        L.orc_reduce_local.argtypes = [vp, vp, sz, ctypes.c_int, ctypes.c_int]
        L.orc_pi.argtypes = [ctypes.c_int] * 3
        L.orc_remap_rank.argtypes = [ctypes.c_uint32, ctypes.c_uint32]
        L.orc_remap_rank.restype = ctypes.c_uint32
        L.orc_get_nu.argtypes = [ctypes.c_uint32, ctypes.c_uint32]
        L.orc_get_nu.restype = ctypes.c_uint32
        L.orc_static_tables.argtypes = [ctypes.c_int, vp, vp, vp]
        L.orc_allreduce.argtypes = [ctypes.c_char_p, ctypes.c_int, sz, ctypes.c_int, ctypes.c_int,
                                    sz, ctypes.c_int, vp, vp, vp]
        L.orc_reduce_scatter.argtypes = [ctypes.c_char_p, ctypes.c_int, vp, ctypes.c_int,
                                         ctypes.c_int, vp, vp, vp]
        L.orc_allgather.argtypes = [ctypes.c_char_p, ctypes.c_int, sz, ctypes.c_int, ctypes.c_int, vp, vp, vp]
        L.orc_reduce.argtypes = [ctypes.c_char_p, ctypes.c_int, sz, ctypes.c_int, ctypes.c_int,
                                 ctypes.c_int, vp, vp, vp]
        _lib = L
    return _lib


def _ptrs(arrs):
    return (ctypes.c_void_p * len(arrs))(*[a.ctypes.data if a is not None else None for a in arrs])


def fill(dtype: str, n: int, seed: int) -> np.ndarray:
    """pico_core's generator (pico_core_utils.c:883-928) with seed `seed`."""
    a = np.zeros(n, dtype=NP_DTYPES[dtype])   # pair types: padding bytes stay 0
    lib().orc_fill(a.ctypes.data, DTYPES[dtype], n, seed)
    return a


def sparsify(x: np.ndarray, dtype: str, rank: int) -> np.ndarray:
    """oracle/ref_golden.c sparsify(): with j = i + rank, zero where j % 3 == 0;
    float / double also -0.0 where j % 5 == 1 and NaN where j % 11 == 2 (later
    rules win) -- inputs on which the logical ops and MAX / MIN show their
    operand semantics"""
    j = np.arange(x.size) + rank
    v = x["v"] if x.dtype.names else x
    v[j % 3 == 0] = 0
    if dtype in ("float", "double", "float_int", "double_int"):
        v[j % 5 == 1] = -0.0
        v[j % 11 == 2] = np.nan
    if dtype in ("c_float_complex", "c_double_complex"):
        v.real[j % 5 == 1] = -0.0
        v.imag[j % 7 == 3] = -0.0
    return x


def inputs(dtype: str, n: int, P: int, seed_base: int = 1234, sparse: bool = False):
    if sparse:
        return [sparsify(fill(dtype, n, seed_base + r), dtype, r) for r in range(P)]
    return [fill(dtype, n, seed_base + r) for r in range(P)]


def reduce_local(inp: np.ndarray, inout: np.ndarray, dtype: str, op: str = "sum") -> None:
    """MPI_Reduce_local(in, inout) with MPICH 3.3.2 semantics (in place on inout)."""
    lib().orc_reduce_local(inp.ctypes.data, inout.ctypes.data, inout.size, DTYPES[dtype], OPS[op])


def remap_rank(P: int, r: int) -> int:
    return int(lib().orc_remap_rank(P, r))


def pi(r: int, s: int, P: int) -> int:
    return int(lib().orc_pi(r, s, P))


def static_tables(P: int):
    n = P.bit_length() - 1
    perm = np.zeros(P, np.int32)
    st = np.zeros(P * n, np.int32)
    rt = np.zeros(P * n, np.int32)
    if lib().orc_static_tables(P, perm.ctypes.data, st.ctypes.data, rt.ctypes.data):
        raise ValueError(P)
    return perm, st.reshape(P, n), rt.reshape(P, n)


def allreduce(algo, sbufs, dtype, op="sum", segsize=0, ref_bugs=False):
    P, n = len(sbufs), sbufs[0].size
    rbufs = [np.zeros(n, dtype=NP_DTYPES[dtype]) for _ in range(P)]
    rets = np.zeros(P, np.int32)
    if lib().orc_allreduce(algo.encode(), P, n, DTYPES[dtype], OPS[op], segsize, int(ref_bugs),
                           _ptrs(sbufs), _ptrs(rbufs), rets.ctypes.data):
        raise ValueError(algo)
    return rbufs, rets.tolist()


def reduce_scatter(algo, sbufs, rcounts, dtype, op="sum"):
    P = len(sbufs)
    rc = np.asarray(rcounts, dtype=np.int32)
    rbufs = [np.zeros(max(int(c), 1), dtype=NP_DTYPES[dtype]) for c in rc]
    rets = np.zeros(P, np.int32)
    if lib().orc_reduce_scatter(algo.encode(), P, rc.ctypes.data, DTYPES[dtype], OPS[op],
                                _ptrs(sbufs), _ptrs(rbufs), rets.ctypes.data):
        raise ValueError(algo)
    return [b[:int(c)] for b, c in zip(rbufs, rc)], rets.tolist()


def reduce(algo, sbufs, dtype, op="sum", root=0):
    P, n = len(sbufs), sbufs[0].size
    rbufs = [np.zeros(n, dtype=NP_DTYPES[dtype]) if r == root else None for r in range(P)]
    rets = np.zeros(P, np.int32)
    if lib().orc_reduce(algo.encode(), P, n, DTYPES[dtype], OPS[op], root,
                        _ptrs(sbufs), _ptrs(rbufs), rets.ctypes.data):
        raise ValueError(algo)
    return rbufs[root], rets.tolist()


def allgather(algo, sbufs, dtype, in_place_rbufs=None):
    """sbufs[r]: rank r's count elements; returns (rbufs (P*count each), rets).
    in_place_rbufs: MPI_IN_PLACE -- these P*count buffers already hold each
    rank's block where the algorithm expects it (copied, not modified)."""
    P = len(sbufs)
    n = sbufs[0].size
    if in_place_rbufs is not None:
        rbufs = [np.array(b, dtype=NP_DTYPES[dtype]).copy() for b in in_place_rbufs]
    else:
        rbufs = [np.zeros(P * n, dtype=NP_DTYPES[dtype]) for _ in range(P)]
    rets = np.zeros(P, np.int32)
    if lib().orc_allgather(algo.encode(), P, n, DTYPES[dtype], int(in_place_rbufs is not None),
                           _ptrs(sbufs), _ptrs(rbufs), rets.ctypes.data):
        raise ValueError(algo)
    return rbufs, rets.tolist()


ERR_ROOT = 7   # MPICH's MPI_ERR_ROOT


def bcast(algo, sbufs, dtype, root=0):
    """bcast latency trees, in place (each rank's buffer = its input); returns
    (buffers after the broadcast, rets).  Message-level replay of the
    reference: every step's transfers are applied in order, a rank forwards
    only what it holds.
      bine_lat / _reversed  libbine_bcast.c:189-279 / :281-371 (root 0 only)
      bine_lat_new / _i_new :373-406 / :408-452 (negabinary partners, any root)
    P = 1 with the _new variants: the reference shifts by -1 (:384, :421) and
    crashes; here the broadcast of one rank is a no-op."""
    P = len(sbufs)
    bufs = [np.array(b, dtype=NP_DTYPES[dtype]).copy() for b in sbufs]
    steps = P.bit_length() - 1
    if P & (P - 1):
        return bufs, [ERR_SIZE] * P
    if algo in ("bine_lat", "bine_lat_reversed"):
        if root != 0:
            return bufs, [ERR_ROOT] * P
        have = {0}
        for s in range(steps):
            ss = steps - s - 1 if algo == "bine_lat_reversed" else s
            moves = [(x, pi(x, ss, P)) for x in sorted(have) if pi(x, ss, P) not in have]
            for src, dst in moves:
                bufs[dst][:] = bufs[src]
            have |= {d for _, d in moves}
        have = [r in have for r in range(P)]
    elif algo in ("bine_lat_new", "bine_lat_i_new"):
        M = 0xAAAAAAAA
        have = [r == root for r in range(P)]
        mask = 1 << (steps - 1) if steps else 0
        while mask > 0:
            lo = (mask << 1) - 1
            moves = []
            for r in range(P):
                nb = (((r - root) % P) + M) & 0xFFFFFFFF ^ M
                partner = (((((nb ^ lo) ^ M) - M) & 0xFFFFFFFF) + root) % P
                lsbs = nb & lo
                if not have[r] and (lsbs == 0 or lsbs == lo):
                    moves.append((partner, r))
            for src, dst in moves:
                assert have[src], (algo, P, root, src, dst)
                bufs[dst][:] = bufs[src]
                have[dst] = True
            mask >>= 1
    else:
        raise ValueError(algo)
    assert all(have), (algo, P, root)
    return bufs, [OK] * P


def _mix64(x):
    x = (x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    x = (x ^ (x >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return x ^ (x >> np.uint64(31))


def digest(a: np.ndarray) -> int:
    """bine_checksum's order-independent digest on the host (sum over i of
    mix64(bits(x[i]) + i * 0x9E3779B97F4A7C15) mod 2^64), in slabs to bound
    memory -- the size-independent form in which full-size oracle outputs are
    compared with the device's (tests/golden/bench_digests.json)."""
    bits_t = {1: np.uint8, 2: np.uint16, 4: np.uint32, 8: np.uint64}[a.dtype.itemsize]
    raw = a.view(bits_t)
    tot = np.uint64(0)
    slab = 1 << 22
    with np.errstate(over="ignore"):
        for s in range(0, a.size, slab):
            bits = raw[s:s + slab].astype(np.uint64)
            idx = np.arange(s, s + bits.size, dtype=np.uint64) * np.uint64(0x9E3779B97F4A7C15)
            tot = tot + _mix64(bits + idx).sum(dtype=np.uint64)
    return int(tot)


def reduce_tree(leaves, dtype: str, op: str = "sum", swap: int = 0) -> np.ndarray:
    """The flat reduce-scatter's tree (bine_reduce_tree) as the literal
    schedule computes it: pairwise MPI_Reduce_local calls level by level,
    v[j] = v[j] (op) v[j + w] (libbine_allreduce.c:888's operand order:
    inout = the left subtree; levels whose bit is set in `swap` keep the right
    subtree as inout, libbine_reduce_scatter.c:1143)."""
    v = [np.array(x, copy=True) for x in leaves]
    w, lvl = 1, 0
    while w < len(v):
        for j in range(0, len(v), 2 * w):
            if (swap >> lvl) & 1:
                reduce_local(v[j], v[j + w], dtype, op)
                v[j] = v[j + w]
            else:
                reduce_local(v[j + w], v[j], dtype, op)
        w, lvl = 2 * w, lvl + 1
    return v[0]


def rs_rcounts(N: int, P: int, kind: str = "even"):
    """Block sizes used by the golden capture (oracle/ref_golden.c)."""
    return [N // P + ((i % 3) if kind == "ragged" else 0) for i in range(P)]
