"""The C ABI: libraries load and export every symbol include/*.h declares
(host-only: no compute call, no GPU needed)."""
import os
import re

import pico_amd
from pico_amd import _lib

INC = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include")


def _declared(header):
    text = open(os.path.join(INC, header)).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return set(re.findall(r"^\s*(?:const\s+)?[\w\s\*]+?\b(\w+)\s*\(", text, flags=re.M)) - {"defined"}


def test_core_library_exports_header():
    pico_amd.lib()
    names = _declared("bine_amd.h")
    assert "bine_allreduce" in names and "bine_reduce_local" in names
    missing = names - _lib.exported_symbols(_lib.CORE)
    assert not missing, missing


def test_dropin_exports_every_libbine_prototype():
    """pico_core's selectors reference every prototype of libbine.h
    (pico_core_utils.c:103-249): the drop-in must export all 41 + the segsize global."""
    names = _declared("libbine_amd.h")
    assert len(names) == 41, len(names)
    syms = _lib.exported_symbols(_lib.SHIM)
    assert not names - syms, names - syms
    import subprocess
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.SHIM], capture_output=True, text=True).stdout
    assert re.search(r" [BD] bine_allreduce_segsize$", out, flags=re.M)


def test_algorithm_names_and_pico_core_selectors():
    L = pico_amd.lib()
    for coll, algos in pico_amd.ALGOS.items():
        for name, code in algos.items():
            assert L.bine_algo_from_name(coll.encode(), name.encode()) == code
            assert L.bine_algo_from_name(coll.encode(), f"{coll}_{name}".encode()) == code
    # pico_core's own selector strings (pico_core_utils.c:104-111, 206-207, 222-230)
    sel = {("allreduce", "bine_bdw_remap_over"): 5, ("allreduce", "recursive_doubling_over"): 0,
           ("allreduce", "bine_block_by_block_any_even"): 7, ("reduce", "bine_bdw_over"): 33,
           ("reduce_scatter", "bine_permute_remap_over"): 22, ("reduce_scatter", "recursive_halving_over"): 16}
    for (coll, s), code in sel.items():
        assert L.bine_algo_from_name(coll.encode(), s.encode()) == code
    assert L.bine_algo_from_name(b"allreduce", b"nope") == -1


def test_dtype_sizes():
    L = pico_amd.lib()
    for name, code in pico_amd.DTYPES.items():
        assert L.bine_dtype_size(code) == _lib.DTYPE_SIZE[name]


def test_op_valid_matches_mpich_table():
    """bine_op_valid (host-only) against the (op, type) pairs MPICH 3.3.2's
    MPI_Reduce_local accepts (probed with it): no bitwise op on float /
    double, MAXLOC / MINLOC exactly on the pair types, SUM / PROD only on the
    complex types"""
    import pico_amd
    from pico_amd._lib import DTYPES, OPS
    lib = pico_amd.lib()
    for d, dv in DTYPES.items():
        for o, ov in OPS.items():
            pair, loc = d in ("float_int", "double_int", "long_int", "2int", "short_int"), o in ("maxloc", "minloc")
            want = pair == loc and not (o in ("band", "bor", "bxor") and d in ("float", "double"))
            if d.startswith("c_"):
                want = o in ("sum", "prod")   # C99 complex: SUM / PROD only
            assert bool(lib.bine_op_valid(dv, ov)) == want, (d, o)
    assert not lib.bine_op_valid(17, 0) and not lib.bine_op_valid(0, 12)


def test_rccl_abi_window_refuses_a_skewed_pair():
    """the RCCL pair the library is built against / runs on
    must lie in the window whose ABI for every type it passes was checked
    (executor.cpp: static_asserts on the header values, bine_rccl_abi_check,
    the creation-time probe); outside it bine_comm_init_rccl refuses, while
    bine_rccl_version stays a reporter and rccl_version() says
    abi_ok."""
    L = pico_amd.lib()
    assert L.bine_rccl_abi_check(22606, 22707) == 0     # torch's runtime, ROCm 7.2's headers
    assert L.bine_rccl_abi_check(22703, 22703) == 0
    err = 5   # BINE_ERR_RCCL (include/bine_amd.h)
    for rt, ct in ((22509, 22707), (22800, 22707), (22606, 22800), (32000, 22707), (22606, 21900)):
        rc = L.bine_rccl_abi_check(rt, ct)
        assert rc != 0, (rt, ct)
        if err is not None:
            assert rc == err
        assert b"skew" in L.bine_last_error()
    # this process's own pair (loading librccl needs no GPU): inside the window
    import ctypes
    rt, ct = ctypes.c_int(), ctypes.c_int()
    assert L.bine_rccl_version(ctypes.byref(rt), ctypes.byref(ct)) == 0, L.bine_last_error()
    assert 22600 <= rt.value <= 22799 and 22600 <= ct.value <= 22799
    v = pico_amd.rccl_version()
    assert v["abi_ok"] is True and v["runtime_code"] == rt.value
