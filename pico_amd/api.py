"""Python mirror of libbine's reduce-family operator interface on MI355X.

Every function named after a libbine entry point (reference include/libbine.h:
30-78) takes the same arguments in the same order --
``allreduce_bine_bdw_remap(sbuf, rbuf, count, dtype, op, comm)`` -- where the
buffers are device tensors (torch, ROCm) or raw device addresses, ``dtype`` is a
libbine element-type name ("float", "double", "int32", ...) or a torch dtype,
``op`` is "sum" | "prod" | "max" | "min" | "land" | "lor" | "lxor" | "band" | "bor" | "bxor" |
"maxloc" | "minloc" (MPICH semantics; bitwise ops on integer types only, the loc ops on
the pair types "float_int" | "double_int" | "long_int" | "2int" | "short_int" only; the
complex types "c_float_complex" | "c_double_complex" under "sum" / "prod" only), and
``comm`` is a :class:`Comm`.
Errors raise :class:`BineError` carrying the status the reference would return
as an MPI error class.  The work runs in libbine_amd.so (HIP kernels + RCCL);
there is no fallback.
"""
from __future__ import annotations

import ctypes
from typing import Optional, Sequence

from . import _lib
from ._lib import ALGOS, DTYPES, OPS, BineError, check, lib

IN_PLACE = "IN_PLACE"   # libbine's MPI_IN_PLACE

_TORCH_DT = None


def _torch_dtypes():
    global _TORCH_DT
    if _TORCH_DT is None:
        import torch
        _TORCH_DT = {torch.float32: "float", torch.float64: "double", torch.int8: "int8",
                     torch.uint8: "uint8", torch.int16: "int16", torch.int32: "int32",
                     torch.int64: "int64"}
    return _TORCH_DT


def _dtype(dtype, *bufs) -> int:
    if dtype is None:
        for b in bufs:
            if hasattr(b, "dtype"):
                dtype = b.dtype
                break
    if not isinstance(dtype, str):
        dtype = _torch_dtypes()[dtype]
    return DTYPES[dtype]


def _ptr(buf):
    if buf is None:
        return None
    if isinstance(buf, str) and buf == IN_PLACE:
        return _lib.IN_PLACE.value
    if hasattr(buf, "data_ptr"):
        return buf.data_ptr()
    return int(buf)


def _stream(stream, comm: Optional["Comm"]):
    if stream is not None:
        return stream if isinstance(stream, int) else getattr(stream, "cuda_stream", stream)
    try:
        import torch
        if torch.cuda.is_available():
            dev = comm.device if comm is not None else torch.cuda.current_device()
            return torch.cuda.current_stream(dev).cuda_stream
    except Exception:  # pragma: no cover
        pass
    return comm.stream if comm is not None else None


class Comm:
    """A bine communicator: one rank of an RCCL communicator (one process per
    GPU) or one virtual rank of an in-process loopback group."""

    def __init__(self, handle: int, kind: str):
        self.handle = ctypes.c_void_p(handle)
        self.kind = kind

    # -- construction --------------------------------------------------------
    @staticmethod
    def unique_id() -> bytes:
        buf = ctypes.create_string_buffer(_lib.UNIQUE_ID_BYTES)
        check(lib().bine_get_unique_id(buf), "bine_get_unique_id")
        return buf.raw

    @classmethod
    def rccl(cls, rank: int, size: int, unique_id: bytes, device: int = 0) -> "Comm":
        h = ctypes.c_void_p()
        idbuf = ctypes.create_string_buffer(unique_id, _lib.UNIQUE_ID_BYTES)
        check(lib().bine_comm_init_rccl(ctypes.byref(h), size, rank, idbuf, device), "bine_comm_init_rccl")
        return cls(h.value, "rccl")

    @classmethod
    def from_torch_distributed(cls, device: int, group=None) -> "Comm":
        """Bootstrap over an initialised torch.distributed group (any backend):
        rank 0 creates the RCCL unique id and broadcasts it."""
        import torch
        import torch.distributed as dist
        rank, size = dist.get_rank(group), dist.get_world_size(group)
        uid = cls.unique_id() if rank == 0 else bytes(_lib.UNIQUE_ID_BYTES)
        t = torch.tensor(list(uid), dtype=torch.uint8)
        if dist.get_backend(group) == "nccl":
            t = t.cuda(device)
        dist.broadcast(t, 0, group=group)
        return cls.rccl(rank, size, bytes(t.cpu().tolist()), device)

    @classmethod
    def loopback(cls, nranks: int, device: int = 0) -> list["Comm"]:
        arr = (ctypes.c_void_p * nranks)()
        check(lib().bine_comm_init_loopback(arr, nranks, device), "bine_comm_init_loopback")
        return [cls(arr[r], "loopback") for r in range(nranks)]

    # -- properties ----------------------------------------------------------
    @property
    def rank(self) -> int:
        return lib().bine_comm_rank(self.handle)

    @property
    def size(self) -> int:
        return lib().bine_comm_size(self.handle)

    @property
    def device(self) -> int:
        return lib().bine_comm_device(self.handle)

    @property
    def stream(self) -> int:
        return lib().bine_comm_stream(self.handle)

    def synchronize(self) -> None:
        check(lib().bine_comm_synchronize(self.handle), "bine_comm_synchronize")

    def set_trees(self, on: bool) -> None:
        """Multi-tree mode (allreduce, P = 4 / 8); collective."""
        check(lib().bine_comm_set_trees(self.handle, int(on)), "bine_comm_set_trees")

    def set_coll_a2a(self, on: bool) -> None:
        """RCCL communicators, relay / trees off: exchanges with one equal-sized
        message to and from every peer as one ncclAllToAllv; bit-identical."""
        check(lib().bine_comm_set_coll_a2a(self.handle, int(on)), "bine_comm_set_coll_a2a")

    def set_coll_ag(self, on: bool) -> None:
        """RCCL communicators: run one-buffer-to-all-peers exchanges (the flat
        allgather phase) as ncclAllGather + device copies; bit-identical."""
        check(lib().bine_comm_set_coll_ag(self.handle, int(on)), "bine_comm_set_coll_ag")

    def set_flat_ag(self, on) -> None:
        """Allreduce (remap / static, power-of-two P): one all-peers allgather
        exchange after the Bine reduce-scatter; bit-identical; collective.
        on = 2: with the flat reduce-scatter, the allgather is cut with its
        chunks (outputs complete chunk by chunk)."""
        check(lib().bine_comm_set_flat_ag(self.handle, int(on)), "bine_comm_set_flat_ag")

    def set_flat_rs(self, on: bool) -> None:
        """Flat reduce-scatter phase (one all-peers exchange + the reference's
        reduction tree in one kernel; bit-identical); collective."""
        check(lib().bine_comm_set_flat_rs(self.handle, int(on)), "bine_comm_set_flat_rs")

    def set_graphs(self, on: bool) -> None:
        """Graph mode (RCCL communicators): capture each (collective, buffers,
        stream) once into a HIP graph and replay it; bit-identical; the
        stream must not be the NULL stream."""
        check(lib().bine_comm_set_graphs(self.handle, int(on)), "bine_comm_set_graphs")

    def fused_calls(self) -> int:
        """large collectives issued as one k_dm_fused launch (bine_comm_fused_calls)"""
        n = lib().bine_comm_fused_calls(self.handle)
        if n < 0:
            check(int(-n), "bine_comm_fused_calls")
        return int(n)

    def graphs_cached(self) -> int:
        """graphs graph mode holds (0: every call so far ran eagerly)"""
        n = lib().bine_comm_graphs_cached(self.handle)
        if n < 0:
            check(int(-n), "bine_comm_graphs_cached")
        return int(n)

    def set_direct(self, on: bool) -> None:
        """RCCL communicators on one node: exchanges through mapped peer memory
        (bine_comm_set_direct); bit-identical.  EVERY call with on=True is
        collective (all ranks, same point: set-up, or the rebuild of a
        transport a timeout disabled on any rank); on=False is local."""
        check(lib().bine_comm_set_direct(self.handle, int(on)), "bine_comm_set_direct")

    def set_direct_wgs(self, wgs: int) -> None:
        """workgroups per message of the direct transport (0 = default;
        bine_comm_set_direct_wgs); local, drops cached graphs"""
        check(lib().bine_comm_set_direct_wgs(self.handle, int(wgs)), "bine_comm_set_direct_wgs")

    def set_direct_tree(self, on) -> None:
        """direct transport: the flat reduce-scatter's trees inside the exchange
        launches (bine_comm_set_direct_tree; -1 = BINE_DIRECT_TREE); every rank
        alike; bit-identical"""
        check(lib().bine_comm_set_direct_tree(self.handle, int(on)), "bine_comm_set_direct_tree")

    def direct_timed_out(self) -> bool:
        """a wait of this rank's direct transport timed out (bine_comm_direct_timed_out)"""
        n = lib().bine_comm_direct_timed_out(self.handle)
        if n < 0:
            check(int(-n), "bine_comm_direct_timed_out")
        return bool(n)

    def direct_ping(self, peer: int, iters: int = 1000) -> float:
        """microseconds per cross-GPU flag round trip with `peer` over the
        direct transport (bine_comm_direct_ping; both ranks call it together)"""
        us = ctypes.c_double(0.0)
        check(lib().bine_comm_direct_ping(self.handle, peer, iters, ctypes.byref(us)), "bine_comm_direct_ping")
        return us.value

    def direct_stamps(self, reset: bool = True):
        """Direct-transport diagnostics (BINE_DIRECT_STAMPS=<records> at setup;
        bine_comm_direct_stamps): numpy uint64 array (n, 4) of per-workgroup
        records -- tag (serial << 32 | kind << 24 | msg << 16 | wg; kind 0 push,
        1 pull, 2 tree), wall_clock64 at entry, wait done, copy done."""
        import numpy as np
        n = ctypes.c_size_t(0)
        check(lib().bine_comm_direct_stamps(self.handle, None, 0, ctypes.byref(n), 0), "bine_comm_direct_stamps")
        out = np.zeros((max(int(n.value), 1), 4), dtype=np.uint64)
        check(lib().bine_comm_direct_stamps(self.handle, out.ctypes.data, int(n.value), ctypes.byref(n),
                                            int(reset)), "bine_comm_direct_stamps")
        return out[:min(int(n.value), out.shape[0])] if n.value else out[:0]

    def set_profile(self, on: bool) -> None:
        """Per-op device timing of the following collectives (bine_comm_set_profile)."""
        check(lib().bine_comm_set_profile(self.handle, int(on)), "bine_comm_set_profile")

    def profile(self):
        """Per-op timing of the latest profiled collective: list of
        {"xchg", "nprims", "bytes", "start_ms", "ms"} in issue order."""
        n = lib().bine_comm_profile(self.handle, None, 0)
        if n < 0:
            raise BineError(int(-n), "bine_comm_profile")
        arr = (_lib.OpTime * max(int(n), 1))()
        n = lib().bine_comm_profile(self.handle, arr, n)
        if n < 0:
            raise BineError(int(-n), "bine_comm_profile")
        return [{f: getattr(arr[k], f) for f, _ in _lib.OpTime._fields_} for k in range(int(n))]

    def set_chunk(self, nbytes: int) -> None:
        """Pipelining chunk in bytes (0 = default 16 MiB); never changes a bit; collective."""
        check(lib().bine_comm_set_chunk(self.handle, nbytes), "bine_comm_set_chunk")

    def set_relay(self, min_part_bytes: int) -> None:
        """Multi-link relay for permutation steps (0 = off); collective."""
        check(lib().bine_comm_set_relay(self.handle, min_part_bytes), "bine_comm_set_relay")

    def destroy(self) -> None:
        if self.handle:
            lib().bine_comm_destroy(self.handle)
            self.handle = ctypes.c_void_p()


# ---- arithmetic boundary ------------------------------------------------------

def reduce_local(inbuf, inoutbuf, count: int, dtype=None, op: str = "sum", stream=None) -> None:
    """MPI_Reduce_local on the GPU: inout = inout (op) in."""
    check(lib().bine_reduce_local(_ptr(inbuf), _ptr(inoutbuf), count, _dtype(dtype, inbuf), OPS[op],
                                  _stream(stream, None)), "bine_reduce_local")


def reduce3(a, b, out, count: int, dtype=None, op: str = "sum", stream=None) -> None:
    """out = b (op) a (out may alias b)."""
    check(lib().bine_reduce3(_ptr(a), _ptr(b), _ptr(out), count, _dtype(dtype, a), OPS[op],
                             _stream(stream, None)), "bine_reduce3")


def fill_pico(buf, count: int, dtype=None, seed: int = 1234, stream=None) -> None:
    """pico_core's rand_r() input distribution, generated on the device."""
    check(lib().bine_fill_pico(_ptr(buf), count, _dtype(dtype, buf), seed, _stream(stream, None)),
          "bine_fill_pico")


def copy(dst, src, nbytes: int, stream=None) -> None:
    """copy_buffer on the device (bine_copy: the k_copy kernel every COPY
    primitive runs)."""
    check(lib().bine_copy(_ptr(dst), _ptr(src), nbytes, _stream(stream, None)), "bine_copy")


def rccl_version() -> dict:
    """{"runtime": code, "compiled": code, ..., "abi_ok"}: the RCCL this process
    maps vs the headers libbine_amd.so was compiled against (NCCL_VERSION
    codes), and whether the pair lies in the checked ABI window -- reported
    also when it does not (communicator creation refuses such a pair)."""
    rt, ct = ctypes.c_int(), ctypes.c_int()
    check(lib().bine_rccl_version(ctypes.byref(rt), ctypes.byref(ct)), "bine_rccl_version")

    def fmt(v):
        return f"{v // 10000}.{v // 100 % 100}.{v % 100}"
    return {"runtime": fmt(rt.value), "compiled": fmt(ct.value), "runtime_code": rt.value,
            "compiled_code": ct.value, "abi_ok": lib().bine_rccl_abi_check(rt.value, ct.value) == 0}


def checksum(buf, count: int, dtype=None, stream=None) -> int:
    out = ctypes.c_uint64()
    check(lib().bine_checksum(_ptr(buf), count, _dtype(dtype, buf), ctypes.byref(out), _stream(stream, None)),
          "bine_checksum")
    return out.value


def set_reduce_tuning(unroll: int = 4, maxblocks: int = 0, nontemporal: int = 0) -> None:
    lib().bine_set_reduce_tuning(unroll, maxblocks, nontemporal)


# ---- generic collectives -------------------------------------------------------

def _algo(coll: str, algo) -> int:
    return algo if isinstance(algo, int) else ALGOS[coll][algo]


def allreduce(algo, sbuf, rbuf, count: int, dtype, op: str, comm: Comm, segsize: int = 0, stream=None) -> None:
    check(lib().bine_allreduce(comm.handle, _algo("allreduce", algo), _ptr(sbuf), _ptr(rbuf), count,
                               _dtype(dtype, rbuf), OPS[op], segsize, _stream(stream, comm)), f"allreduce_{algo}")


def reduce_scatter(algo, sbuf, rbuf, rcounts: Sequence[int], dtype, op: str, comm: Comm, stream=None) -> None:
    rc = (ctypes.c_int * len(rcounts))(*rcounts)
    check(lib().bine_reduce_scatter(comm.handle, _algo("reduce_scatter", algo), _ptr(sbuf), _ptr(rbuf), rc,
                                    _dtype(dtype, rbuf), OPS[op], _stream(stream, comm)), f"reduce_scatter_{algo}")


def allreduce_staged(algo, host_sbuf, host_rbuf, dev_sbuf, dev_rbuf, count: int, dtype, op: str, comm: Comm,
                     h2d_stream, d2h_stream, segsize: int = 0, chunk_bytes: int = 0, stream=None) -> None:
    """bine_allreduce_staged: host buffers (page-locked) staged through the
    device buffers piece by piece, pipelined with the collective; synchronize
    `stream` to complete the call."""
    check(lib().bine_allreduce_staged(comm.handle, _algo("allreduce", algo), _ptr(host_sbuf), _ptr(host_rbuf),
                                      _ptr(dev_sbuf), _ptr(dev_rbuf), count, _dtype(dtype, dev_rbuf), OPS[op],
                                      segsize, chunk_bytes, _stream(h2d_stream, comm), _stream(d2h_stream, comm),
                                      _stream(stream, comm)), f"allreduce_staged_{algo}")


def reduce_scatter_staged(algo, host_sbuf, host_rbuf, dev_sbuf, dev_rbuf, rcounts: Sequence[int], dtype, op: str,
                          comm: Comm, h2d_stream, d2h_stream, chunk_bytes: int = 0, stream=None) -> None:
    """bine_reduce_scatter_staged (see allreduce_staged)."""
    rc = (ctypes.c_int * len(rcounts))(*rcounts)
    check(lib().bine_reduce_scatter_staged(comm.handle, _algo("reduce_scatter", algo), _ptr(host_sbuf),
                                           _ptr(host_rbuf), _ptr(dev_sbuf), _ptr(dev_rbuf), rc,
                                           _dtype(dtype, dev_rbuf), OPS[op], chunk_bytes,
                                           _stream(h2d_stream, comm), _stream(d2h_stream, comm),
                                           _stream(stream, comm)), f"reduce_scatter_staged_{algo}")


def reduce(algo, sbuf, rbuf, count: int, dtype, op: str, root: int, comm: Comm, stream=None) -> None:
    check(lib().bine_reduce(comm.handle, _algo("reduce", algo), _ptr(sbuf), _ptr(rbuf), count,
                            _dtype(dtype, sbuf if rbuf is None else rbuf), OPS[op], root, _stream(stream, comm)),
          f"reduce_{algo}")


# ---- loopback group drivers (all virtual ranks of one device) -------------------

def _ptrs(bufs):
    return (ctypes.c_void_p * len(bufs))(*[_ptr(b) for b in bufs])


def loopback_allreduce(comms, algo, sbufs, rbufs, count, dtype, op="sum", segsize=0):
    st = (ctypes.c_int * len(comms))()
    hs = (ctypes.c_void_p * len(comms))(*[c.handle.value for c in comms])
    rc = lib().bine_loopback_run_allreduce(hs, len(comms), _algo("allreduce", algo), _ptrs(sbufs), _ptrs(rbufs),
                                           count, _dtype(dtype, rbufs[0]), OPS[op], segsize, st)
    return rc, list(st)


def loopback_reduce_scatter(comms, algo, sbufs, rbufs, rcounts, dtype, op="sum"):
    st = (ctypes.c_int * len(comms))()
    hs = (ctypes.c_void_p * len(comms))(*[c.handle.value for c in comms])
    rcs = (ctypes.c_int * len(rcounts))(*rcounts)
    rc = lib().bine_loopback_run_reduce_scatter(hs, len(comms), _algo("reduce_scatter", algo), _ptrs(sbufs),
                                                _ptrs(rbufs), rcs, _dtype(dtype, rbufs[0]), OPS[op], st)
    return rc, list(st)


def loopback_reduce(comms, algo, sbufs, rbufs, count, dtype, op="sum", root=0):
    st = (ctypes.c_int * len(comms))()
    hs = (ctypes.c_void_p * len(comms))(*[c.handle.value for c in comms])
    rc = lib().bine_loopback_run_reduce(hs, len(comms), _algo("reduce", algo), _ptrs(sbufs), _ptrs(rbufs),
                                        count, _dtype(dtype, sbufs[0]), OPS[op], root, st)
    return rc, list(st)


# ---- schedule introspection ------------------------------------------------------

def plan(coll: str, algo, nranks: int, rank: int, count: int = 0, rcounts=None, root: int = 0,
         esz: int = 4, segsize: int = 0, in_place: bool = False):
    """Rank `rank`'s primitive list (host only).  Returns (prims, tmp_elems) or
    raises BineError with the reference's error status."""
    a = _algo(coll, algo)
    rc = (ctypes.c_int * nranks)(*(rcounts or [0] * nranks))
    tmp = (ctypes.c_uint64 * 3)()
    n = lib().bine_plan(a, nranks, rank, count, rc, root, esz, segsize, int(in_place), None, 0, tmp)
    if n < 0:
        raise BineError(int(-n), f"plan {coll}_{algo}")
    arr = (_lib.Prim * max(int(n), 1))()
    lib().bine_plan(a, nranks, rank, count, rc, root, esz, segsize, int(in_place), arr, n, tmp)
    prims = [{f: getattr(arr[k], f) for f, _ in _lib.Prim._fields_ } for k in range(int(n))]
    for p in prims:
        p["type"] = _lib.PRIM_NAMES[p["type"]]
    return prims, list(tmp)


def schedule(coll: str, algo, nranks: int, rank: int, count: int = 0, rcounts=None, root: int = 0,
             esz: int = 4, segsize: int = 0, in_place: bool = False, chunk_bytes: int = 0,
             relay_min_bytes: int = 0, info: bool = False, trees: bool = False, flat_ag: bool = False,
             flat_rs: bool = False):
    """The executor's two-stream issue schedule of rank `rank` (host only).
    Returns (ops, c_join, final_wait); ops[i] = {"xchg", "wait", "prims"}.
    With info=True a 4th item: {"tmp_elems": [TMP0..2], "stage_elems": relay staging}."""
    a = _algo(coll, algo)
    rc = (ctypes.c_int * nranks)(*(rcounts or [0] * nranks))
    cj, fw, ws = ctypes.c_int(), ctypes.c_int64(), (ctypes.c_uint64 * 4)()
    args = (a, nranks, rank, count, rc, root, esz, segsize, int(in_place), chunk_bytes, relay_min_bytes,
            int(trees) | (2 if flat_ag else 0) | (4 if flat_rs else 0) | (8 if flat_ag == 2 else 0))
    n = lib().bine_plan_schedule(*args, None, 0, ctypes.byref(cj), ctypes.byref(fw), ws)
    if n < 0:
        raise BineError(int(-n), f"schedule {coll}_{algo}")
    arr = (_lib.SchedEntry * max(int(n), 1))()
    lib().bine_plan_schedule(*args, arr, n, ctypes.byref(cj), ctypes.byref(fw), ws)
    ops = []
    for k in range(int(n)):
        e = arr[k]
        p = {f: getattr(e.prim, f) for f, _ in _lib.Prim._fields_ }
        p["type"] = _lib.PRIM_NAMES[p["type"]]
        if not ops or e.op != len(ops) - 1:
            ops.append({"xchg": bool(e.xchg), "wait": int(e.wait), "prims": []})
        ops[-1]["prims"].append(p)
    if info:
        return ops, bool(cj.value), int(fw.value), {"tmp_elems": [int(x) for x in ws[:3]],
                                                     "stage_elems": int(ws[3])}
    return ops, bool(cj.value), int(fw.value)


def dm_tree_plan(coll: str, algo, nranks: int, rank: int, count: int = 0, rcounts=None, esz: int = 4,
                 in_place: bool = False, chunk_bytes: int = 0, flat_ag=False, flat_rs: bool = False,
                 slot: int = 16 << 20, merge: int = 3, dtype="float", op: str = "sum"):
    """The direct transport's fused-tree decisions for rank `rank`'s issue
    schedule (bine_plan_dm_trees, host only): (host, defer) per op -- host[i]
    = the exchange whose launch evaluates tree op i (-1: not fused), defer[i]
    = exchange i's receives are pulled by the next exchange."""
    a = _algo(coll, algo)
    rc = (ctypes.c_int * nranks)(*(rcounts or [0] * nranks))
    mode = (2 if flat_ag else 0) | (4 if flat_rs else 0) | (8 if flat_ag == 2 else 0)
    args = (a, nranks, rank, count, rc, 0, esz, int(in_place), chunk_bytes, mode, slot, merge, _dtype(dtype),
            OPS[op])
    n = lib().bine_plan_dm_trees(*args, None, None, 0)
    if n < 0:
        raise BineError(int(-n), f"dm_tree_plan {coll}_{algo}")
    host, defer = (ctypes.c_int32 * max(int(n), 1))(), (ctypes.c_int32 * max(int(n), 1))()
    lib().bine_plan_dm_trees(*args, host, defer, n)
    return list(host[:n]), list(defer[:n])


def dm_fused_plan(coll: str, algo, nranks: int, rank: int, count: int = 0, rcounts=None, esz: int = 4,
                  in_place: bool = False, chunk_bytes: int = 0, flat_ag=False, flat_rs: bool = False,
                  slot: int = 64 << 20, dtype="float", op: str = "sum", small: bool = False) -> int:
    """k_dm_fused launches the direct transport issues for rank `rank`'s call
    (bine_plan_dm_fused, host only; fused trees on): 0 = the per-exchange
    launches instead."""
    a = _algo(coll, algo)
    rc = (ctypes.c_int * nranks)(*(rcounts or [0] * nranks))
    mode = (2 if flat_ag else 0) | (4 if flat_rs else 0) | (8 if flat_ag == 2 else 0)
    n = lib().bine_plan_dm_fused(a, nranks, rank, count, rc, 0, esz, int(in_place), chunk_bytes, mode, slot,
                                 _dtype(dtype), OPS[op], int(small))
    if n < 0:
        raise BineError(int(-n), f"dm_fused_plan {coll}_{algo}")
    return int(n)


def dm_fused_msgs(coll: str, algo, nranks: int, rank: int, count: int = 0, rcounts=None, esz: int = 4,
                  in_place: bool = False, chunk_bytes: int = 0, flat_ag=False, flat_rs: bool = False,
                  slot: int = 64 << 20, dtype="float", op: str = "sum", small: bool = False):
    """(launches, [(launch, push, peer, bytes), ...]) of the one-launch form
    (bine_plan_dm_fused_msgs): the messages in sequence-number order"""
    a = _algo(coll, algo)
    rc = (ctypes.c_int * nranks)(*(rcounts or [0] * nranks))
    mode = (2 if flat_ag else 0) | (4 if flat_rs else 0) | (8 if flat_ag == 2 else 0)
    args = (a, nranks, rank, count, rc, 0, esz, int(in_place), chunk_bytes, mode, slot, _dtype(dtype), OPS[op],
            int(small))
    n = ctypes.c_int64(0)
    nl = lib().bine_plan_dm_fused_msgs(*args, None, 0, ctypes.byref(n))
    if nl < 0:
        raise BineError(int(-nl), f"dm_fused_msgs {coll}_{algo}")
    buf = (ctypes.c_uint64 * max(4 * n.value, 4))()
    lib().bine_plan_dm_fused_msgs(*args, buf, n.value, ctypes.byref(n))
    return int(nl), [tuple(int(x) for x in buf[4 * k:4 * k + 4]) for k in range(n.value)]


def stage_plan(coll: str, algo, nranks: int, rank: int, count: int = 0, rcounts=None, esz: int = 4,
               segsize: int = 0, in_place: bool = False, chunk_bytes: int = 0, flat_ag=False, flat_rs: bool = False):
    """The host staging of rank `rank`'s schedule (bine_plan_stage; host only):
    (h2d, d2h, h2d_wait) with h2d / d2h = {op: [(lo, hi), ...]} element ranges
    copied before / after op, h2d_wait = [newest op whose h2d batch op i waits
    for, or -1]."""
    a = _algo(coll, algo)
    rc = (ctypes.c_int * nranks)(*(rcounts or [0] * nranks))
    mode = (2 if flat_ag else 0) | (4 if flat_rs else 0) | (8 if flat_ag == 2 else 0)
    res = []
    for kind, w in ((0, 3), (1, 3), (2, 2)):
        args = (a, nranks, rank, count, rc, 0, esz, segsize, int(in_place), chunk_bytes, mode, kind)
        n = lib().bine_plan_stage(*args, None, 0)
        if n < 0:
            raise BineError(int(-n), f"stage_plan {coll}_{algo}")
        arr = (ctypes.c_uint64 * max(int(n) * w, 1))()
        lib().bine_plan_stage(*args, arr, n)
        if kind < 2:
            d = {}
            for k in range(int(n)):
                d.setdefault(int(arr[3 * k]), []).append((int(arr[3 * k + 1]), int(arr[3 * k + 2])))
            res.append(d)
        else:
            res.append([ctypes.c_int64(arr[2 * k + 1]).value for k in range(int(n))])
    return tuple(res)


def reduce_batch(ins, inouts, counts, dtype, op: str = "sum", stream=None) -> int:
    """inouts[k][:counts[k]] = inouts[k] (op) ins[k], all windows in one launch.
    Returns the status (BINE_ERR_ARG = 1 when windows are not co-aligned)."""
    n = len(ins)
    c = (ctypes.c_size_t * n)(*counts)
    b = _ptrs(inouts)
    return lib().bine_reduce_batch(n, _ptrs(ins), b, b, c, _dtype(dtype, inouts[0]), OPS[op], _stream(stream, None))


def reduce_tree(leaves, out, count: int, dtype, op: str = "sum", stream=None) -> int:
    """out[:count] = the reduction tree over the leaf buffers (tree order,
    len 2/4/8/16) in one launch (bine_reduce_tree).  Returns the status."""
    return lib().bine_reduce_tree(len(leaves), _ptrs(leaves), _ptr(out), count, _dtype(dtype, out), OPS[op],
                                  _stream(stream, None))


def exchange(comm: Comm, sends=(), recvs=(), stream=None) -> None:
    """One group of P2P transfers (bine_exchange): sends / recvs are
    (peer, buffer, nbytes) triples; receives match the peers' sends in size
    and posting order."""
    ns, nr = len(sends), len(recvs)
    sp = (ctypes.c_int * max(ns, 1))(*[p for p, _, _ in sends])
    sb = (ctypes.c_void_p * max(ns, 1))(*[_ptr(b) for _, b, _ in sends])
    sz = (ctypes.c_size_t * max(ns, 1))(*[n for _, _, n in sends])
    rp = (ctypes.c_int * max(nr, 1))(*[p for p, _, _ in recvs])
    rb = (ctypes.c_void_p * max(nr, 1))(*[_ptr(b) for _, b, _ in recvs])
    rz = (ctypes.c_size_t * max(nr, 1))(*[n for _, _, n in recvs])
    check(lib().bine_exchange(comm.handle, ns, sp, sb, sz, nr, rp, rb, rz, _stream(stream, comm)), "exchange")


def vendor_allreduce(sbuf, rbuf, count: int, dtype, op: str, comm: Comm, stream=None) -> None:
    """RCCL's own ncclAllReduce on the same communicator (bine_vendor_allreduce):
    a measurement baseline beside the Bine path, not a libbine algorithm."""
    check(lib().bine_vendor_allreduce(comm.handle, _ptr(sbuf), _ptr(rbuf), count, _dtype(dtype, rbuf), OPS[op],
                                      _stream(stream, comm)), "vendor_allreduce")


def allgather(algo, sbuf, rbuf, count: int, dtype, comm: Comm, stream=None) -> None:
    """count = elements per rank; rbuf holds comm.size * count elements."""
    check(lib().bine_allgather(comm.handle, _algo("allgather", algo), _ptr(sbuf), _ptr(rbuf), count,
                               _dtype(dtype, rbuf), _stream(stream, comm)), f"allgather_{algo}")


def loopback_allgather(comms, algo, sbufs, rbufs, count, dtype):
    st = (ctypes.c_int * len(comms))()
    hs = (ctypes.c_void_p * len(comms))(*[c.handle.value for c in comms])
    rc = lib().bine_loopback_run_allgather(hs, len(comms), _algo("allgather", algo), _ptrs(sbufs), _ptrs(rbufs),
                                           count, _dtype(dtype, rbufs[0]), st)
    return rc, list(st)


def bcast(algo, buf, count: int, dtype, root: int, comm: Comm, stream=None) -> None:
    """root's `count` elements of buf reach every rank (in place)."""
    check(lib().bine_bcast(comm.handle, _algo("bcast", algo), _ptr(buf), count, _dtype(dtype, buf), root,
                           _stream(stream, comm)), f"bcast_{algo}")


def loopback_bcast(comms, algo, bufs, count, dtype, root):
    st = (ctypes.c_int * len(comms))()
    hs = (ctypes.c_void_p * len(comms))(*[c.handle.value for c in comms])
    rc = lib().bine_loopback_run_bcast(hs, len(comms), _algo("bcast", algo), _ptrs(bufs), count,
                                       _dtype(dtype, bufs[0]), root, st)
    return rc, list(st)


def gather(algo, sbuf, rbuf, count: int, dtype, root: int, comm: Comm, stream=None) -> None:
    """every rank's `count` elements of sbuf land in block r of the root's rbuf
    (P * count elements; rbuf may be None elsewhere)."""
    check(lib().bine_gather(comm.handle, _algo("gather", algo), _ptr(sbuf), _ptr(rbuf), count,
                            _dtype(dtype, sbuf), root, _stream(stream, comm)), f"gather_{algo}")


def scatter(algo, sbuf, rbuf, count: int, dtype, root: int, comm: Comm, stream=None) -> None:
    """block r of the root's sbuf (P * count elements; sbuf may be None
    elsewhere) lands in rank r's rbuf (`count` elements)."""
    check(lib().bine_scatter(comm.handle, _algo("scatter", algo), _ptr(sbuf), _ptr(rbuf), count,
                             _dtype(dtype, rbuf), root, _stream(stream, comm)), f"scatter_{algo}")


def alltoall(algo, sbuf, rbuf, count: int, dtype, comm: Comm, stream=None) -> None:
    """block j of rank r's sbuf lands in block r of rank j's rbuf (both P * count
    elements)."""
    check(lib().bine_alltoall(comm.handle, _algo("alltoall", algo), _ptr(sbuf), _ptr(rbuf), count,
                              _dtype(dtype, rbuf), _stream(stream, comm)), f"alltoall_{algo}")


def _loopback(fn, coll, comms, algo, sbufs, rbufs, count, dtype, *root):
    st = (ctypes.c_int * len(comms))()
    hs = (ctypes.c_void_p * len(comms))(*[c.handle.value for c in comms])
    ref = next(b for b in list(rbufs) + list(sbufs) if b is not None)
    rc = fn(hs, len(comms), _algo(coll, algo), _ptrs(sbufs), _ptrs(rbufs), count, _dtype(dtype, ref), *root, st)
    return rc, list(st)


def loopback_gather(comms, algo, sbufs, rbufs, count, dtype, root):
    return _loopback(lib().bine_loopback_run_gather, "gather", comms, algo, sbufs, rbufs, count, dtype, root)


def loopback_scatter(comms, algo, sbufs, rbufs, count, dtype, root):
    return _loopback(lib().bine_loopback_run_scatter, "scatter", comms, algo, sbufs, rbufs, count, dtype, root)


def loopback_alltoall(comms, algo, sbufs, rbufs, count, dtype):
    return _loopback(lib().bine_loopback_run_alltoall, "alltoall", comms, algo, sbufs, rbufs, count, dtype)


# ---- libbine-named entry points (include/libbine.h:30-78) --------------------------

def _mk_ar(name):
    def f(sbuf, rbuf, count, dtype, op, comm, stream=None, segsize: int = 0):
        allreduce(name, sbuf, rbuf, count, dtype, op, comm, segsize=segsize, stream=stream)
    f.__name__ = "allreduce_" + name
    f.__doc__ = f"allreduce_{name} (libbine_allreduce.c) on MI355X."
    return f


def _mk_rs(name):
    def f(sbuf, rbuf, rcounts, dtype, op, comm, stream=None):
        reduce_scatter(name, sbuf, rbuf, rcounts, dtype, op, comm, stream=stream)
    f.__name__ = "reduce_scatter_" + name
    f.__doc__ = f"reduce_scatter_{name} (libbine_reduce_scatter.c) on MI355X."
    return f


def _mk_rd(name):
    def f(sbuf, rbuf, count, dtype, op, root, comm, stream=None):
        reduce(name, sbuf, rbuf, count, dtype, op, root, comm, stream=stream)
    f.__name__ = "reduce_" + name
    f.__doc__ = f"reduce_{name} (libbine_reduce.c) on MI355X."
    return f


def _mk_ag(name):
    def f(sbuf, rbuf, count, dtype, comm, stream=None):
        allgather(name, sbuf, rbuf, count, dtype, comm, stream=stream)
    f.__name__ = "allgather_" + name
    f.__doc__ = f"allgather_{name} (libbine_allgather.c) on MI355X."
    return f


def _mk_bc(name):
    def f(buf, count, dtype, root, comm, stream=None):
        bcast(name, buf, count, dtype, root, comm, stream=stream)
    f.__name__ = "bcast_" + name
    f.__doc__ = f"bcast_{name} (libbine_bcast.c) on MI355X."
    return f


ENTRY_POINTS = {}
for _n in ALGOS["allreduce"]:
    ENTRY_POINTS["allreduce_" + _n] = _mk_ar(_n)
for _n in ALGOS["reduce_scatter"]:
    ENTRY_POINTS["reduce_scatter_" + _n] = _mk_rs(_n)
for _n in ALGOS["reduce"]:
    ENTRY_POINTS["reduce_" + _n] = _mk_rd(_n)
for _n in ALGOS["allgather"]:
    ENTRY_POINTS["allgather_" + _n] = _mk_ag(_n)
for _n in ALGOS["bcast"]:
    ENTRY_POINTS["bcast_" + _n] = _mk_bc(_n)
ENTRY_POINTS["alltoall_bine"] = lambda sbuf, rbuf, count, dtype, comm, stream=None: \
    alltoall("bine", sbuf, rbuf, count, dtype, comm, stream=stream)
ENTRY_POINTS["gather_bine"] = lambda sbuf, rbuf, count, dtype, root, comm, stream=None: \
    gather("bine", sbuf, rbuf, count, dtype, root, comm, stream=stream)
ENTRY_POINTS["scatter_bine"] = lambda sbuf, rbuf, count, dtype, root, comm, stream=None: \
    scatter("bine", sbuf, rbuf, count, dtype, root, comm, stream=stream)
globals().update(ENTRY_POINTS)

__all__ = ["Comm", "BineError", "IN_PLACE", "schedule", "dm_fused_plan", "dm_fused_msgs", "reduce_local", "reduce3", "fill_pico", "checksum", "copy",
           "rccl_version",
           "set_reduce_tuning", "allreduce", "reduce_scatter", "reduce", "loopback_allreduce",
           "loopback_reduce_scatter", "loopback_reduce", "plan", "allgather", "loopback_allgather", "bcast", "loopback_bcast", "reduce_batch",
           "gather", "scatter", "alltoall", "loopback_gather", "loopback_scatter", "loopback_alltoall",
           "exchange", "vendor_allreduce", "reduce_tree", "allreduce_staged", "reduce_scatter_staged",
           "stage_plan", "dm_tree_plan"] + list(ENTRY_POINTS)
