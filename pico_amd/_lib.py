"""ctypes binding of libbine_amd.so (include/bine_amd.h).

The product path is the HIP library; there is no Python or CPU fallback.  If the
shared library is missing this module raises at import time.
"""
from __future__ import annotations

import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIBDIR = os.path.join(HERE, "lib")
CORE = os.path.join(LIBDIR, "libbine_amd.so")
SHIM = os.path.join(LIBDIR, "libbine.so")

# include/bine_amd.h enums
DTYPES = {"int8": 0, "uint8": 1, "int16": 2, "uint16": 3, "int32": 4, "uint32": 5,
          "int64": 6, "uint64": 7, "float": 8, "double": 9,
          # MPI's (value, index) pair types, MAXLOC / MINLOC only
          "float_int": 10, "double_int": 11, "long_int": 12, "2int": 13, "short_int": 14,
          # C99 complex, SUM / PROD only
          "c_float_complex": 15, "c_double_complex": 16}
DTYPE_SIZE = {"int8": 1, "uint8": 1, "int16": 2, "uint16": 2, "int32": 4, "uint32": 4,
              "int64": 8, "uint64": 8, "float": 4, "double": 8,
              "float_int": 8, "double_int": 16, "long_int": 16, "2int": 8, "short_int": 8,
              "c_float_complex": 8, "c_double_complex": 16}
OPS = {"sum": 0, "prod": 1, "max": 2, "min": 3, "land": 4, "band": 5, "lor": 6, "bor": 7, "lxor": 8, "bxor": 9,
       "maxloc": 10, "minloc": 11}
STATUS = {0: "SUCCESS", 1: "ERR_ARG", 2: "ERR_SIZE", 3: "ERR_NO_MEM", 4: "ERR_HIP", 5: "ERR_RCCL",
          6: "ERR_UNSUPPORTED", 7: "ERR_INTERNAL", 8: "ERR_ROOT", 9: "ERR_COUNT"}
ALGOS = {
    "allreduce": {"recursivedoubling": 0, "ring": 1, "rabenseifner": 2, "bine_lat": 3,
                  "bine_bdw_static": 4, "bine_bdw_remap": 5, "bine_bdw_remap_segmented": 6,
                  "bine_block_by_block_any_even": 7},
    "reduce_scatter": {"recursivehalving": 16, "recursive_distance_doubling": 17, "ring": 18,
                       "butterfly": 19, "bine_static": 20, "bine_send_remap": 21,
                       "bine_permute_remap": 22, "bine_block_by_block": 23,
                       "bine_block_by_block_any_even": 24},
    "reduce": {"bine_lat": 32, "bine_bdw": 33},
    "allgather": {"recursivedoubling": 48, "k_bruck": 49, "ring": 50, "sparbit": 51,
                  "bine_block_by_block": 52, "bine_block_by_block_any_even": 53,
                  "bine_permute_static": 54, "bine_send_static": 55, "bine_permute_remap": 56,
                  "bine_send_remap": 57, "bine_2_blocks": 58, "bine_2_blocks_dtype": 59},
    # libbine_bcast.c: the latency trees and (round 5) the bandwidth algorithms
    "bcast": {"scatter_allgather": 64, "bine_lat": 65, "bine_lat_reversed": 66, "bine_lat_new": 67, "bine_lat_i_new": 68,
              "bine_bdw_static": 69, "bine_bdw_remap": 70},
    # libbine_alltoall.c, libbine_gather.c, libbine_scatter.c (round 5)
    "alltoall": {"bine": 80},
    "gather": {"bine": 81},
    "scatter": {"bine": 82},
}
IN_PLACE = ctypes.c_void_p(-1 & 0xFFFFFFFFFFFFFFFF)
UNIQUE_ID_BYTES = 128


class Prim(ctypes.Structure):
    _fields_ = [("type", ctypes.c_int32), ("group", ctypes.c_int32), ("peer", ctypes.c_int32),
                ("flags", ctypes.c_int32), ("src_buf", ctypes.c_int32), ("dst_buf", ctypes.c_int32),
                ("aux_buf", ctypes.c_int32), ("pos", ctypes.c_int32), ("src_off", ctypes.c_uint64),
                ("dst_off", ctypes.c_uint64), ("aux_off", ctypes.c_uint64), ("count", ctypes.c_uint64)]


class SchedEntry(ctypes.Structure):
    _fields_ = [("op", ctypes.c_int32), ("xchg", ctypes.c_int32), ("wait", ctypes.c_int64), ("prim", Prim)]


class OpTime(ctypes.Structure):
    _fields_ = [("xchg", ctypes.c_int32), ("nprims", ctypes.c_int32), ("bytes", ctypes.c_uint64),
                ("start_ms", ctypes.c_float), ("ms", ctypes.c_float)]


PRIM_NAMES = {1: "SEND", 2: "RECV", 3: "REDUCE", 4: "REDUCE3", 5: "COPY", 6: "REDUCE_TREE"}


class BineError(RuntimeError):
    def __init__(self, status: int, what: str = ""):
        self.status = status
        msg = STATUS.get(status, str(status))
        detail = ""
        try:
            detail = lib().bine_last_error().decode()
        except Exception:  # pragma: no cover
            pass
        super().__init__(f"{what}: {msg} {detail}".strip())


_lib = None


def lib():
    """Load libbine_amd.so (build it with __graft_entry__.build())."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(CORE):
        raise ImportError(f"{CORE} not built -- run __graft_entry__.build() (make -C pico_amd/csrc)")
    # One HIP runtime per process: torch (ROCm wheel) bundles its own
    # libamdhip64 / libhsa-runtime64 / librccl.  Loaded first, they satisfy this
    # library's DT_NEEDED by soname and the whole process shares them; loaded
    # after /opt/rocm's copies (this library first, torch later) the process
    # would hold two HIP runtimes and one of them sees no device.  So torch, if
    # installed, is imported before the library is mapped.  The RCCL version
    # in use is reported by bine_rccl_version() (and recorded by bench.py).
    try:
        import torch  # noqa: F401
    except ImportError:  # pragma: no cover -- plain ctypes use without torch: /opt/rocm's runtime
        pass
    L = ctypes.CDLL(CORE)
    vp, sz, i, u32, u64 = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_uint32, ctypes.c_uint64
    sigs = {
        "bine_status_string": ([i], ctypes.c_char_p),
        "bine_last_error": ([], ctypes.c_char_p),
        "bine_dtype_size": ([i], sz),
        "bine_op_valid": ([i, i], i),
        "bine_algo_from_name": ([ctypes.c_char_p, ctypes.c_char_p], i),
        "bine_algo_name": ([i], ctypes.c_char_p),
        "bine_set_reduce_tuning": ([i, i, i], i),
        "bine_reduce_local": ([vp, vp, sz, i, i, vp], i),
        "bine_reduce3": ([vp, vp, vp, sz, i, i, vp], i),
        "bine_fill_pico": ([vp, sz, i, u32, vp], i),
        "bine_copy": ([vp, vp, sz, vp], i),
        "bine_rccl_version": ([ctypes.POINTER(i), ctypes.POINTER(i)], i),
        "bine_rccl_abi_check": ([i, i], i),
        "bine_dm_fit_residency": ([ctypes.POINTER(i), i, ctypes.POINTER(i), i], i),
        "bine_comm_direct_timed_out": ([vp], i),
        "bine_comm_direct_ping": ([vp, i, i, ctypes.POINTER(ctypes.c_double)], i),
        "bine_dropin_defaults": ([i, ctypes.POINTER(i), ctypes.POINTER(i), ctypes.POINTER(i)], i),
        "bine_dm_launch_cap": ([i, i, i, i, i], i),
        "bine_dm_residency_cap": ([i, i, i, i], i),
        "bine_checksum": ([vp, sz, i, ctypes.POINTER(u64), vp], i),
        "bine_get_unique_id": ([vp], i),
        "bine_comm_init_rccl": ([ctypes.POINTER(vp), i, i, vp, i], i),
        "bine_comm_init_loopback": ([vp, i, i], i),
        "bine_comm_destroy": ([vp], i),
        "bine_comm_rank": ([vp], i),
        "bine_comm_size": ([vp], i),
        "bine_comm_device": ([vp], i),
        "bine_comm_stream": ([vp], vp),
        "bine_comm_synchronize": ([vp], i),
        "bine_allreduce": ([vp, i, vp, vp, sz, i, i, sz, vp], i),
        "bine_reduce_scatter": ([vp, i, vp, vp, vp, i, i, vp], i),
        "bine_reduce": ([vp, i, vp, vp, sz, i, i, i, vp], i),
        "bine_allgather": ([vp, i, vp, vp, sz, i, vp], i),
        "bine_reduce_batch": ([i, vp, vp, vp, vp, i, i, vp], i),
        "bine_reduce_tree": ([i, vp, vp, ctypes.c_size_t, i, i, vp], i),
        "bine_loopback_run_allgather": ([vp, i, i, vp, vp, sz, i, vp], i),
        "bine_bcast": ([vp, i, vp, sz, i, i, vp], i),
        "bine_loopback_run_bcast": ([vp, i, i, vp, sz, i, i, vp], i),
        "bine_gather": ([vp, i, vp, vp, sz, i, i, vp], i),
        "bine_scatter": ([vp, i, vp, vp, sz, i, i, vp], i),
        "bine_alltoall": ([vp, i, vp, vp, sz, i, vp], i),
        "bine_loopback_run_gather": ([vp, i, i, vp, vp, sz, i, i, vp], i),
        "bine_loopback_run_scatter": ([vp, i, i, vp, vp, sz, i, i, vp], i),
        "bine_loopback_run_alltoall": ([vp, i, i, vp, vp, sz, i, vp], i),
        "bine_loopback_run_allreduce": ([vp, i, i, vp, vp, sz, i, i, sz, vp], i),
        "bine_loopback_run_reduce_scatter": ([vp, i, i, vp, vp, vp, i, i, vp], i),
        "bine_loopback_run_reduce": ([vp, i, i, vp, vp, sz, i, i, i, vp], i),
        "bine_plan": ([i, i, i, sz, vp, i, sz, sz, i, vp, ctypes.c_int64, ctypes.POINTER(u64)],
                      ctypes.c_int64),
        "bine_comm_set_relay": ([vp, sz], i),
        "bine_comm_set_trees": ([vp, i], i),
        "bine_comm_set_chunk": ([vp, sz], i),
        "bine_comm_set_flat_ag": ([vp, i], i),
        "bine_comm_set_coll_ag": ([vp, i], i),
        "bine_comm_set_coll_a2a": ([vp, i], i),
        "bine_comm_set_flat_rs": ([vp, i], i),
        "bine_comm_set_graphs": ([vp, i], i),
        "bine_comm_graphs_cached": ([vp], ctypes.c_int64),
        "bine_comm_fused_calls": ([vp], ctypes.c_int64),
        "bine_comm_set_direct": ([vp, i], i),
        "bine_comm_set_direct_wgs": ([vp, i], i),
        "bine_comm_set_direct_tree": ([vp, i], i),
        "bine_comm_direct_stamps": ([vp, vp, sz, ctypes.POINTER(sz), i], i),
        "bine_comm_set_profile": ([vp, i], i),
        "bine_comm_profile": ([vp, vp, ctypes.c_int64], ctypes.c_int64),
        "bine_exchange": ([vp, i, vp, vp, vp, i, vp, vp, vp, vp], i),
        "bine_vendor_allreduce": ([vp, vp, vp, sz, i, i, vp], i),
        "bine_plan_schedule": ([i, i, i, sz, vp, i, sz, sz, i, sz, sz, i, vp, ctypes.c_int64, ctypes.POINTER(ctypes.c_int),
                                ctypes.POINTER(ctypes.c_int64), vp], ctypes.c_int64),
        "bine_plan_stage": ([i, i, i, sz, vp, i, sz, sz, i, sz, i, i, vp, ctypes.c_int64], ctypes.c_int64),
        "bine_plan_dm_fused": ([i, i, i, sz, vp, i, sz, i, sz, i, sz, i, i, i], i),
        "bine_plan_dm_fused_msgs": ([i, i, i, sz, vp, i, sz, i, sz, i, sz, i, i, i, vp, ctypes.c_int64,
                                     ctypes.POINTER(ctypes.c_int64)], ctypes.c_int64),
        "bine_plan_dm_trees": ([i, i, i, sz, vp, i, sz, i, sz, i, sz, i, i, i, vp, vp, ctypes.c_int64],
                               ctypes.c_int64),
        "bine_allreduce_staged": ([vp, i, vp, vp, vp, vp, sz, i, i, sz, sz, vp, vp, vp], i),
        "bine_reduce_scatter_staged": ([vp, i, vp, vp, vp, vp, vp, i, i, sz, vp, vp, vp], i),
    }
    for name, (args, res) in sigs.items():
        f = getattr(L, name)
        f.argtypes = args
        f.restype = res
    _lib = L
    return L


def check(status: int, what: str) -> None:
    if status != 0:
        raise BineError(status, what)


def exported_symbols(path: str):
    """Dynamic symbols a shared library defines (host-side check, no GPU)."""
    import subprocess
    out = subprocess.run(["nm", "-D", "--defined-only", path], capture_output=True, text=True, check=True).stdout
    return {line.split()[-1] for line in out.splitlines() if " T " in line}
