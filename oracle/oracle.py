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


def _source_sha256() -> str:
    import hashlib
    h = hashlib.sha256()
    for f in ("bine_oracle.c", "bine_oracle.h"):
        with open(os.path.join(_HERE, f), "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()


def build() -> str:
    """liboracle.so, built from exactly the sources beside it: its stamp
    (liboracle.so.sha256, written by oracle/Makefile) must name their sha256.
    Missing or stale: compiled (gcc) in the build container -- where
    /root/reference is mounted, __graft_entry__.build() runs -- and an error
    anywhere else: on the GPU box the checker is the one
    built here and shipped with the tree, never silently rebuilt."""
    stamp = _LIB + ".sha256"
    want = _source_sha256()
    try:
        with open(stamp) as f:
            ok = os.path.exists(_LIB) and f.read().strip() == want
    except OSError:
        ok = False
    if not ok:
        if not os.path.isdir("/root/reference"):
            raise RuntimeError("oracle/liboracle.so is missing or was not built from the bine_oracle.c / .h beside "
                               "it, and this is not the build container: the checker is built by "
                               "__graft_entry__.build() and shipped, never rebuilt where the tests run")
        subprocess.run(["make", "-s", "-B", "-C", _HERE, "liboracle.so"], check=True)
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


ERR_COUNT = 2   # MPICH's MPI_ERR_COUNT
BC_BDW = ("scatter_allgather", "bine_bdw_static", "bine_bdw_remap")


class _Stuck(Exception):
    pass


def _replay(P, bufs, programs, leftover=None):
    """Run one generator per rank -- a line-by-line restatement of a reference
    function -- with MPI's point-to-point semantics: a send is buffered (its
    bytes are snapshotted when posted, as MPI_Send / MPI_Isend of an unmodified
    buffer deliver them), a receive takes the oldest message of its
    (source, destination) pair, places it at its offset and reports its
    element count (MPI_Get_count); a message longer than the receive's count
    is MPI_ERR_TRUNCATE and ends the replay.  Yields: ("send", dst, off, n),
    ("recv", src, off, maxn) -> n on the rank's one buffer, or ("send", dst,
    view) / ("recv", src, view) -> n naming the bytes of any buffer.  A rank's return value is its status.
    Raises _Stuck when no rank can move (the reference would hang)."""
    import collections
    q = collections.defaultdict(collections.deque)
    gens = [programs[r]() for r in range(P)]
    rets = [None] * P
    pending = [None] * P   # the op a rank waits on
    val = [None] * P
    while any(x is None for x in rets):
        moved = False
        for r in range(P):
            while rets[r] is None:
                if pending[r] is None:
                    try:
                        pending[r] = gens[r].send(val[r])
                    except StopIteration as e:
                        rets[r] = e.value if e.value is not None else OK
                        moved = True
                        break
                    val[r] = None
                    moved = True
                op = pending[r]
                if len(op) == 3:
                    # ("send", dst, view) / ("recv", src, view): a program over
                    # several buffers names the bytes itself (_sl bounds-checks)
                    if op[0] == "send":
                        q[(r, op[1])].append(np.array(op[2]))
                        pending[r] = None
                        moved = True
                        continue
                    if not q[(op[1], r)]:
                        break
                    m = q[(op[1], r)].popleft()
                    if m.size > op[2].size:
                        raise ValueError("MPI_ERR_TRUNCATE")
                    op[2][:m.size] = m
                    val[r] = m.size
                    pending[r] = None
                    moved = True
                    continue
                if op[0] == "send":
                    _, dst, off, n = op
                    if off + n > bufs[r].size:
                        raise ValueError("a send reads past the buffer")
                    q[(r, dst)].append(np.array(bufs[r][off:off + n]))
                    pending[r] = None
                    moved = True
                    continue
                _, src, off, maxn = op
                if not q[(src, r)]:
                    break
                m = q[(src, r)].popleft()
                if m.size > maxn:
                    raise ValueError("MPI_ERR_TRUNCATE")
                if off + m.size > bufs[r].size:
                    raise ValueError("a receive writes past the buffer")
                bufs[r][off:off + m.size] = m
                val[r] = m.size
                pending[r] = None
                moved = True
        if not moved:
            raise _Stuck()
    if leftover is not None:   # messages sent and never received
        leftover.extend(k for k, v in q.items() if v)
    return rets


def _bc_scatter_allgather(P, count, root, bufs):
    """bcast_scatter_allgather, libbine_bcast.c:42-187 (binomial-tree scatter,
    recursive-doubling allgather with the non-power-of-two forwarding)"""
    def prog(rank):
        def g():
            if P < 2:
                return OK
            if count < P:
                return ERR_COUNT
            u = lambda x: x % (1 << 64)   # the reference's size_t arithmetic (it wraps)
            vrank = (rank - root + P) % P
            sc = (count + P - 1) // P
            curr = count if rank == root else 0
            recv_count = 0
            mask = 1
            while mask < P:                                         # :73-91
                if vrank & mask:
                    parent = (rank - mask + P) % P
                    recv_count = u(count - vrank * sc)
                    if recv_count == 0:
                        curr = 0
                    else:
                        curr = yield ("recv", parent, vrank * sc, recv_count)
                    break
                mask <<= 1
            mask >>= 1
            while mask > 0:                                         # :93-106
                if vrank + mask < P:
                    send_count = u(curr - sc * mask)
                    if send_count > 0:
                        yield ("send", (rank + mask) % P, sc * (vrank + mask), send_count)
                        curr = u(curr - send_count)
                mask >>= 1
            rem = u(count - vrank * sc)                             # :112-115
            curr = min(sc, rem)
            mask = 1
            while mask < P:                                         # :117-171
                vremote = vrank ^ mask
                remote = (vremote + root) % P
                vtr = (vrank // mask) * mask
                vrtr = (vremote // mask) * mask
                if vremote < P:
                    recv_count = u(count - vrtr * sc)
                    yield ("send", remote, vtr * sc, curr)
                    recv_count = yield ("recv", remote, vrtr * sc, recv_count)
                    curr += recv_count
                if vrtr + mask > P:
                    nad = P - vtr - mask
                    off = sc * (vtr + mask)
                    rh = mask >> 1
                    while rh > 0:
                        vrem = vrank ^ rh
                        rem_r = (vrem + root) % P
                        tree_root = (vrank // (rh << 1)) * (rh << 1)
                        if vrem > vrank and vrank < tree_root + nad and vrem >= tree_root + nad:
                            yield ("send", rem_r, off, recv_count)
                        elif vrem < vrank and vrem < tree_root + nad and vrank >= tree_root + nad:
                            recv_count = yield ("recv", rem_r, off, count)
                            curr += recv_count
                        rh >>= 1
                mask <<= 1
            return OK
        return g
    return [prog(r) for r in range(P)]


def _bc_bine_bdw_static(P, count, root, bufs):
    """bcast_bine_bdw_static, libbine_bcast.c:462-647 (static-table scatter,
    mirrored allgather)"""
    steps = P.bit_length() - 1
    tables = static_tables(P) if P >= 2 and P == 1 << steps else None

    def prog(rank):
        def g():
            if P < 2:
                return OK
            if count < P:
                return ERR_COUNT
            if P != 1 << steps:
                return ERR_SIZE
            if root != 0:
                return ERR_ROOT
            received = [False] * P
            received[root] = True
            recv_step = -1
            step = 0
            while step < steps and not received[rank]:              # :519-530
                for proc in range(P):
                    if not received[proc]:
                        continue
                    dest = pi(proc, step, P)
                    received[dest] = True
                    if dest == rank:
                        recv_step = step
                        break
                step += 1
            split = count % P
            small = count // P
            big = small + (1 if split else 0)
            _, sb, rb = tables
            s_bm, r_bm = list(sb[rank]), list(rb[rank])

            def cnt(b, w):
                return w * big if b + w <= split else w * small if b >= split else w * small + (split - b)

            def offs(b):
                return b * big if b <= split else b * small + split
            w = P >> 1
            for step in range(steps):                               # :556-587
                if rank != root and recv_step == step:
                    yield ("recv", pi(rank, step, P), offs(r_bm[step]), cnt(r_bm[step], w))
                if recv_step < step:
                    yield ("send", pi(rank, step, P), offs(s_bm[step]), cnt(s_bm[step], w))
                w >>= 1
            w = 1
            for step in range(steps - 1, -1, -1):                   # :606-632
                dest = pi(rank, step, P)
                if recv_step != step:
                    yield ("send", dest, offs(r_bm[step]), cnt(r_bm[step], w))
                if not recv_step < step:
                    yield ("recv", dest, offs(s_bm[step]), cnt(s_bm[step], w))
                w <<= 1
            return OK
        return g
    return [prog(r) for r in range(P)]


def _bc_bine_bdw_remap(P, count, root, bufs):
    """bcast_bine_bdw_remap, libbine_bcast.c:649-760 (negabinary-remapped
    scatter + allgather); root 0 only (:650 asserts)"""
    steps = P.bit_length() - 1
    nb2b = lambda x: ((x ^ 0xAAAAAAAA) - 0xAAAAAAAA) & 0xFFFFFFFF   # negabinary_to_binary

    def sgn(v):
        return v - (1 << 32) if v >= 1 << 31 else v

    def prog(rank):
        def g():
            per, rem = count // P, count % P
            displs = [per * i + (i if i < rem else rem) for i in range(P)]
            rc = [per + (1 if i < rem else 0) for i in range(P)]
            mask = 1
            inv = 1 << (steps - 1) if steps else 0
            bfm = ~(inv - 1) if inv else -1
            rr = remap_rank(P, rank)
            recv_mask = inv << 1
            if rank != root:
                recv_mask = rr & -rr
            recvd = rank == root

            def partner():
                d = sgn(nb2b((mask << 1) - 1))
                return (rank + d) % P if rank % 2 == 0 else (rank - d) % P
            while mask < P:                                         # :689-716
                pt = partner()
                sf = remap_rank(P, pt) & bfm
                sl = sf + inv - 1
                scount = displs[sl] - displs[sf] + rc[sl]
                rf = rr & bfm
                rl = rf + inv - 1
                rcount = displs[rl] - displs[rf] + rc[rl]
                if recvd:
                    yield ("send", pt, displs[sf], scount)
                elif inv == recv_mask or pt == root:
                    yield ("recv", pt, displs[rf], rcount)
                    recvd = True
                mask <<= 1
                inv >>= 1
                bfm >>= 1
            mask >>= 1                                              # :719-751
            inv = 1
            bfm = -1
            while mask > 0:
                pt = partner()
                rp = None if inv < recv_mask else pt
                sp = None if inv == recv_mask else pt
                if sp is not None:
                    sf = rr & bfm
                    sl = sf + inv - 1
                    yield ("send", sp, displs[sf], displs[sl] - displs[sf] + rc[sl])
                if rp is not None:
                    rf = remap_rank(P, rp) & bfm
                    rl = rf + inv - 1
                    yield ("recv", rp, displs[rf], displs[rl] - displs[rf] + rc[rl])
                mask >>= 1
                inv <<= 1
                bfm <<= 1
            return OK
        return g
    return [prog(r) for r in range(P)]


def bcast_bdw(algo, sbufs, dtype, root=0):
    """the bandwidth bcasts (libbine_bcast.c:42, :462, :649), in place on each
    rank's own input: (buffers after the broadcast, rets), by message-level
    replay of the reference (_replay).  Where the reference crashes or hangs
    (scatter_allgather's size_t counts wrap when a block starts past the
    buffer's end, and a send then reads past it; bine_bdw_remap at root != 0
    or non-power-of-two P): "crash" in every ret."""
    P = len(sbufs)
    bufs = [np.array(b, dtype=NP_DTYPES[dtype]).copy() for b in sbufs]
    n = bufs[0].size if P else 0
    if algo == "bine_bdw_remap" and (root != 0 or P & (P - 1)):
        return bufs, ["crash"] * P
    progs = {"scatter_allgather": _bc_scatter_allgather, "bine_bdw_static": _bc_bine_bdw_static,
             "bine_bdw_remap": _bc_bine_bdw_remap}[algo](P, n, root, bufs)
    try:
        rets = _replay(P, bufs, progs)
    except (_Stuck, ValueError):
        return bufs, ["crash"] * P
    return bufs, rets


# ---- gather / scatter / alltoall (libbine_gather.c, _scatter.c, _alltoall.c) ----
_M32 = 0xFFFFFFFF


def _b2nb(b):
    """binary_to_negabinary (libbine_utils.h:509-513): int32 -> uint32"""
    return _M32 if b > 0x55555555 else ((0xAAAAAAAA + b) & _M32) ^ 0xAAAAAAAA


def _nb2b(n):
    """negabinary_to_binary (libbine_utils.h:515-518): uint32 -> int32"""
    v = ((0xAAAAAAAA ^ (n & _M32)) - 0xAAAAAAAA) & _M32
    return v - (1 << 32) if v >= 1 << 31 else v


def _log2c(v):
    """log_2 (libbine_utils.h:279-288): ceil(log2(v))"""
    return (v - 1).bit_length() if v > 1 else 0


def _nb_in_range(x, nbits):
    """in_range (libbine_utils.h:524-526) over the smallest / largest
    negabinary values of nbits digits (:47-50)"""
    lo = -sum(1 << i for i in range(1, nbits, 2))
    hi = sum(1 << i for i in range(0, nbits, 2))
    return lo <= x <= hi


def _remap_distance_doubling(num):
    """remap_distance_doubling (libbine_utils.h:601-609)"""
    num &= _M32
    out = 0
    while num > 0:
        k = num.bit_length() - 1
        out ^= 1 << k
        num = (num ^ ((1 << (k + 1)) - 1)) & _M32
    return out


class _OOB(ValueError):
    """the reference reads or writes past a buffer (undefined: it may crash or
    run on with heap bytes)"""


def _sl(buf, lo, hi):
    """buf[lo:hi] in elements -- a view; a range past the buffer is the
    reference reading / writing out of bounds (raised, not clipped)"""
    if buf is None:
        raise _Crash()
    if lo < 0 or hi > buf.size or hi < lo:
        raise _OOB()
    return buf[lo:hi]


def _uninit(n, dtype):
    """a malloc'd temporary of the reference: zeros here; None (undefined) in a
    symbolic run on object arrays (tests/rooted_util.defined)"""
    return np.full(n, None, object) if dtype == object else np.zeros(n, dtype)


class _Crash(Exception):
    """the reference aborts (an assert) or dereferences NULL here"""


def _gather_progs(P, n, root, sbufs, rbuf_root):
    """gather_bine, libbine_gather.c:16-96: blocks gathered into a P-block
    buffer (the root's rbuf, a temporary elsewhere), each rank extending its
    resident run up or down at alternate steps (direction from the REAL rank's
    parity, :33-36) and sending the whole run to its negabinary partner once
    its low bits stop matching (:45-57)"""
    def prog(rank):
        def g():
            rb = rbuf_root if rank == root else _uninit(P * n, sbufs[rank].dtype)
            _sl(rb, rank * n, rank * n + n)[:] = sbufs[rank][:n]          # :28
            lo = hi = rank
            vrank = (rank - root) % P
            ext = 1 if rank % 2 == 0 else -1
            mask = 1
            while mask < P:
                nbv = _b2nb(vrank)
                partner = (_nb2b(nbv ^ ((mask << 1) - 1)) + root) % P      # :39-40
                mlsb = (mask << 2) - 1
                lsbs = nbv & mlsb
                equal = lsbs == 0 or lsbs == mlsb
                if not equal or ((mask << 1) >= P and rank != root):       # :45-57
                    if hi >= lo:
                        yield ("send", partner, _sl(rb, lo * n, (hi + 1) * n))
                    else:
                        yield ("send", partner, _sl(rb, lo * n, P * n))
                        yield ("send", partner, _sl(rb, 0, (hi + 1) * n))
                    break
                if ext == 1:                                                # :59-69
                    rs, re = (hi + 1) % P, (hi + mask) % P
                    hi = re
                else:
                    re, rs = (lo - 1) % P, (lo - mask) % P
                    lo = rs
                if re >= rs:                                                # :70-80
                    yield ("recv", partner, _sl(rb, rs * n, (re + 1) * n))
                else:
                    yield ("recv", partner, _sl(rb, rs * n, P * n))
                    yield ("recv", partner, _sl(rb, 0, (re + 1) * n))
                ext = -ext
                mask <<= 1
            return OK
        return g
    return [prog(r) for r in range(P)]


def _scatter_progs(P, n, root, sbuf_root, rbufs):
    """scatter_bine, libbine_scatter.c:14-151: the gather's tree run backwards
    -- resident block range [min, max] from the gather's end state
    (:49-55), halved at every step; a non-root receives its subtree's blocks
    once into a temporary (a leaf straight into rbuf, :110-126) and forwards
    halves from there (relative block indices)"""
    L = _log2c(P)

    def prog(rank):
        def g():
            if P == 1:
                raise _Crash()   # mask = 1 << (log_2(1) - 1): a negative shift (:57)
            vrank = (rank - root) % P
            hd = 1 if rank % 2 == 0 else -1
            if L % 2 == 0:
                hd = -hd
            full = (1 << L) - 1
            if rank % 2 == 0:                                               # :49-55
                maxr = ((rank + 0x55555555) & full) % P
                minr = ((rank - 0xAAAAAAAA) & full) % P
            else:
                minr = ((rank - 0x55555555) & full) % P
                maxr = ((rank + 0xAAAAAAAA) & full) % P
            mask = 1 << (L - 1)
            off = rank
            recvd, leaf, sb = False, False, None
            if rank == root:
                recvd, sb = True, sbuf_root
            vnb = _b2nb(vrank)
            while mask > 0:
                partner = (_nb2b(vnb ^ ((mask << 1) - 1)) + root) % P      # :69-70
                mlsb = (mask << 1) - 1
                lsbs = vnb & mlsb
                equal = lsbs == 0 or lsbs == mlsb
                ts, te = minr, (minr + mask - 1) % P                         # :75-78
                bs, be = (te + 1) % P, maxr
                if hd == 1:
                    ss, se, rs, re = bs, be, ts, te
                    maxr = (maxr - mask) % P
                else:
                    ss, se, rs, re = ts, te, bs, be
                    minr = (minr + mask) % P
                if recvd:                                                    # :95-104
                    if sb is None:
                        raise _Crash()
                    if se >= ss:
                        yield ("send", partner, _sl(sb, ss * n, (se + 1) * n))
                    else:
                        yield ("send", partner, _sl(sb, ss * n, P * n))
                        yield ("send", partner, _sl(sb, 0, (se + 1) * n))
                elif equal:                                                  # :105-137
                    nb = (re - rs + 1) % P
                    if rs == re:
                        rb, leaf = rbufs[rank], True
                    else:
                        sb = rb = _uninit(n * nb, rbufs[rank].dtype)
                        minr, maxr = 0, nb - 1
                        off = (rank - rs) % P
                    if re >= rs:
                        yield ("recv", partner, _sl(rb, 0, n * nb))
                    else:
                        yield ("recv", partner, _sl(rb, 0, n * (P - rs)))
                        yield ("recv", partner, _sl(rb, n * (P - rs), n * (P - rs) + n * (re + 1)))
                    recvd = True
                mask >>= 1
                hd = -hd
            if not leaf:                                                     # :142-144
                if sb is None:
                    raise _Crash()
                rbufs[rank][:n] = _sl(sb, off * n, off * n + n)
            return OK
        return g
    return [prog(r) for r in range(P)]


def _alltoall_progs(P, n, sbufs, rbufs):
    """alltoall_bine, libbine_alltoall.c:14-147: log2(P) butterfly steps with
    the negabinary partner; each step moves to rbuf the blocks whose
    remapped destination falls in the partner's half (:71-94), compacts the
    kept ones to the front of the temporary and receives the partner's into
    its second half (:100-102); a final permutation by
    remap_distance_doubling puts every source's block in place (:121-139)"""
    L = _log2c(P)

    def prog(rank):
        def g():
            tmp = np.array(sbufs[rank][:P * n])
            rb = rbufs[rank]
            resident = list(range(P))
            nres = P
            inv = 1 << (L - 1) if L else 0
            bfm = ~(inv - 1)
            mask = 1
            while mask < P:
                d = _nb2b((mask << 1) - 1)
                partner = (rank + d) % P if rank % 2 == 0 else (rank - d) % P
                mins = remap_rank(P, partner) & bfm
                maxs = mins + inv - 1
                nsend = nkeep = 0
                nxt = []
                for i in range(P):                                           # :71-94
                    block = resident[i % nres]
                    if mins <= remap_rank(P, block) <= maxs:
                        _sl(rb, nsend * n, nsend * n + n)[:] = tmp[i * n:(i + 1) * n]
                        nsend += 1
                    else:
                        if i != nkeep:
                            tmp[nkeep * n:(nkeep + 1) * n] = tmp[i * n:(i + 1) * n]
                        nkeep += 1
                        nxt.append(block)
                if nkeep != P // 2 or nsend != P // 2:
                    raise _Crash()   # :95-96 assert
                nres //= 2
                yield ("send", partner, _sl(rb, 0, nsend * n))             # :100-102 Sendrecv
                yield ("recv", partner, _sl(tmp, (P // 2) * n, (P // 2) * n + nsend * n))
                resident[:nres] = nxt[:nres]
                mask <<= 1
                inv >>= 1
                bfm >>= 1
            for i in range(P):                                               # :121-139
                rot = (i - rank) % P if rank % 2 == 0 else (rank - i) % P
                rep = _b2nb(rot) if _nb_in_range(rot, L) else _b2nb(rot - P)
                idx = _remap_distance_doubling(rep)
                _sl(rb, i * n, (i + 1) * n)[:] = _sl(tmp, idx * n, (idx + 1) * n)
            return OK
        return g
    return [prog(r) for r in range(P)]


def _run_rooted(P, progs):
    """rets of a rooted replay: "hang" (a deadlock), "crash" (an assert, a
    NULL dereference, MPI_ERR_TRUNCATE -- fatal under MPICH's default
    handler), "oob" (a read or write past a buffer: undefined), "dangling"
    (completes but leaves a message unreceived, which MPICH delivers to the
    next call's receive from that rank); else the MPI return codes"""
    left = []
    try:
        rets = _replay(P, None, progs, left)
    except _Stuck:
        return ["hang"] * P
    except _OOB:
        return ["oob"] * P
    except (ValueError, _Crash):
        return ["crash"] * P
    return ["dangling"] * P if left else rets


def gather(sbufs, dtype, root=0):
    """gather_bine by message-level replay: (the root's P * n buffer, rets);
    where the reference does not complete cleanly every ret says why
    (_run_rooted)"""
    P, n = len(sbufs), sbufs[0].size
    out = np.zeros(P * n, NP_DTYPES[dtype])
    rets = _run_rooted(P, _gather_progs(P, n, root, sbufs, out))
    return out, rets


def scatter(sbuf_root, P, dtype, root=0):
    """scatter_bine by message-level replay: sbuf_root holds P blocks of n;
    (every rank's n-element rbuf, rets)"""
    n = sbuf_root.size // P
    rbufs = [np.zeros(n, NP_DTYPES[dtype]) for _ in range(P)]
    rets = _run_rooted(P, _scatter_progs(P, n, root, np.array(sbuf_root), rbufs))
    return rbufs, rets


def alltoall(sbufs, dtype):
    """alltoall_bine by message-level replay: sbufs[r] holds P blocks of n
    (block j for rank j); (every rank's P * n rbuf, rets)"""
    P = len(sbufs)
    n = sbufs[0].size // P
    rbufs = [np.zeros(P * n, NP_DTYPES[dtype]) for _ in range(P)]
    rets = _run_rooted(P, _alltoall_progs(P, n, sbufs, rbufs))
    return rbufs, rets


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
