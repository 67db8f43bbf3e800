#!/usr/bin/env python3
"""Capture golden vectors from the REAL reference libbine (test infrastructure).

Runs ``oracle/_ref/ref_golden`` (built by ``make -C oracle ref`` from the sources
under /root/reference, against the image's MPICH 3.3.2) under ``mpiexec -n P``
and writes:

* ``tests/golden/index.json.gz`` -- one record per (collective, algorithm, op,
  dtype, P, N, segsize, rcounts kind): per-rank return codes, output lengths and
  SHA-256 digests of the outputs;
* ``tests/golden/outputs.npz`` -- the full per-rank outputs of the small cases
  (concatenated over ranks, raw bytes as uint8).

Inputs are not stored: they are regenerated from ``seed_base + rank`` with
pico_core's generator (pico_core/pico_core_utils.c:883-928); the ``fill`` cases
pin that generator itself.  This script needs /root/reference and is run by hand
in the build container only; the fixtures it writes are what travels.
"""
from __future__ import annotations

import gzip
import hashlib
import itertools
import json
import os
import shutil
import subprocess
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "oracle", "_ref", "ref_golden")
OUT = os.path.join(ROOT, "tests", "golden")
MPI = "/opt/conda/bin"
SEED = 1234
ESZ = {"float": 4, "double": 8, "int8": 1, "int16": 2, "int32": 4, "int64": 8, "uint8": 1,
       "float_int": 8, "double_int": 16, "long_int": 16, "2int": 8, "short_int": 8,
       "c_float_complex": 8, "c_double_complex": 16}
CPLX_DT = ["c_float_complex", "c_double_complex"]
# MPI's pair types whose size equals their extent: the reference's copy_buffer
# copies MPI_Type_size x count bytes (libbine_utils.h:176-190), so for the
# padded ones (double_int, long_int, short_int: size 12 / 12 / 6 < extent 16 /
# 16 / 8) its outputs are wrong or it crashes -- no vector to pin against
PAIR_DT = ["float_int", "2int"]

SMALL_N = [1, 2, 7, 8, 13, 64, 333]
MID_N = [4096, 65537]
ALL_DT = ["float", "double", "int32", "int64", "int8", "uint8", "int16"]
FEW_DT = ["float", "int64"]

AR_BINE = ["bine_bdw_remap", "bine_bdw_static", "bine_lat", "bine_block_by_block_any_even"]
AR_CLASSIC = ["recursivedoubling", "ring", "rabenseifner"]
AR_NONPOW2 = {"recursivedoubling", "ring", "rabenseifner", "bine_lat",
              "bine_bdw_remap_segmented", "bine_block_by_block_any_even",
              "bine_bdw_remap", "bine_bdw_static"}  # the last two return MPI_ERR_ARG
RS_BINE = ["bine_permute_remap", "bine_send_remap", "bine_static", "bine_block_by_block",
           "bine_block_by_block_any_even"]
RS_CLASSIC = ["recursivehalving", "recursive_distance_doubling", "ring", "butterfly"]
# reduce_scatter algorithms that honour per-block rcounts (displs); permute_remap
# copies block i into the slot of block remap(i) and needs equal blocks.
RS_RAGGED_OK = {"recursivehalving", "recursive_distance_doubling", "ring", "butterfly",
                "bine_static", "bine_send_remap", "bine_block_by_block",
                "bine_block_by_block_any_even"}
# non-power-of-two sizes: these hang in the reference -- skipped
RS_NONPOW2 = {"recursivehalving", "ring", "butterfly", "bine_block_by_block_any_even",
              "bine_static", "recursive_distance_doubling"}


def run_case(P, coll, algo, op, segsize, rk, dtypes, ns, timeout=120):
    tmp = tempfile.mkdtemp(prefix="golden_")
    env = dict(os.environ, PATH=MPI + ":" + os.environ.get("PATH", ""))
    cmd = [os.path.join(MPI, "mpiexec"), "-n", str(P), BIN, tmp, coll, algo, op, str(segsize),
           rk, str(SEED), ",".join(dtypes), ",".join(str(n) for n in ns)]
    try:
        p = subprocess.run(cmd, env=env, capture_output=True, timeout=timeout)
        failed = p.returncode != 0
    except subprocess.TimeoutExpired:
        failed = True
    recs = []
    for dt in dtypes:
        for n in ns:
            rets, outs = [], []
            for r in range(P):
                path = os.path.join(tmp, f"{dt}.N{n}.r{r}.bin")
                raw = open(path, "rb").read() if os.path.exists(path) else b""
                if len(raw) < 16:   # missing, or cut short by a crash of the reference
                    rets = None
                    break
                ret, outn = np.frombuffer(raw[:16], dtype=np.int64)
                rets.append(int(ret))
                outs.append(raw[16:16 + int(outn) * ESZ[dt]])
            recs.append((dt, n, rets, outs, failed))
    shutil.rmtree(tmp, ignore_errors=True)
    return recs


AG_ALGOS = ["recursivedoubling", "k_bruck", "ring", "sparbit", "bine_block_by_block",
            "bine_block_by_block_any_even", "bine_permute_static", "bine_send_static",
            "bine_permute_remap", "bine_send_remap", "bine_2_blocks", "bine_2_blocks_dtype"]


def allgather_jobs():
    """the allgather family, N = elements per rank"""
    jobs = []
    for P in (1, 2, 3, 4, 5, 6, 8):
        for a in AG_ALGOS:
            jobs.append((P, "allgather", a, "sum", 0, "even", ["float", "int64", "int8"], [1, 2, 7, 64, 333, 4099],
                         True))
    jobs.append((16, "allgather", "bine_permute_remap", "sum", 0, "even", ["float"], [5, 1000], True))
    jobs.append((16, "allgather", "bine_send_static", "sum", 0, "even", ["float"], [5, 1000], True))
    jobs.append((16, "allgather", "sparbit", "sum", 0, "even", ["float"], [5], True))
    jobs.append((16, "allgather", "bine_2_blocks", "sum", 0, "even", ["float"], [5], True))
    return jobs


LOGIC_OPS = ["land", "lor", "lxor"]
BIT_OPS = ["band", "bor", "bxor"]
LOGIC_DT = ["float", "double", "int32", "int8", "uint8"]
BIT_DT = ["int64", "int32", "int16", "int8", "uint8"]


def bcast_jobs():
    """bcast latency trees (libbine_bcast.c:189-452): in place on each rank's
    own input; rcounts "root<k>" = root k ("even" = root 0); non-power-of-two
    P pins the MPI_ERR_SIZE returns, root != 0 the MPI_ERR_ROOT ones"""
    jobs = []
    for P in (1, 2, 3, 4, 6, 8, 16):
        for a in ("bine_lat", "bine_lat_reversed", "bine_lat_new", "bine_lat_i_new"):
            roots = sorted({r for r in (1, P - 1, P // 2) if 0 < r < P})
            for rk in ["even"] + [f"root{r}" for r in roots]:
                jobs.append((P, "bcast", a, "sum", 0, rk, ["float", "int64", "int8"], [1, 7, 333, 4099], True))
    return jobs


BC_BDW = ("scatter_allgather", "bine_bdw_static", "bine_bdw_remap")


def bcast_bdw_jobs():
    """the bandwidth bcasts (libbine_bcast.c:42, :462, :649 -- widening past
    SURVEY.md 8(f)): scatter + allgather, in place on each rank's own input;
    counts below P (MPI_ERR_COUNT), at and around P and multiples of it,
    larger ones; scatter_allgather at every root, bine_bdw_static also at a
    root != 0 (MPI_ERR_ROOT) and non-power-of-two P (MPI_ERR_SIZE),
    bine_bdw_remap root 0 only (it asserts, :650)"""
    jobs = []
    for P in (1, 2, 3, 4, 5, 6, 8, 16):
        ns = sorted({1, 3, P, P + 1, 2 * P, 2 * P + 1, 3 * P - 1, 13, 64, 333, 4099})
        for a in BC_BDW:
            if a == "bine_bdw_remap" and P & (P - 1):
                continue   # non-power-of-two P: the reference's remap_rank is undefined there
            roots = ["even"]
            if a != "bine_bdw_remap":
                roots += [f"root{r}" for r in sorted({r for r in (1, P - 1, P // 2) if 0 < r < P})]
            for rk in roots:
                jobs.append((P, "bcast", a, "sum", 0, rk, ["float", "int64", "int8"], ns, True))
    return jobs


ROOTED = ("gather", "scatter", "alltoall")


def _replay_hangs(O, coll, P, root):
    """the oracle's message-level replay of the reference deadlocks here"""
    n = 1
    sb = [np.arange(n if coll == "gather" else n * P, dtype=np.int32) for _ in range(P)]
    progs = (O._gather_progs(P, n, root, sb, np.zeros(P * n, np.int32)) if coll == "gather" else
             O._scatter_progs(P, n, root, sb[root], [np.zeros(n, np.int32) for _ in range(P)])
             if coll == "scatter" else O._alltoall_progs(P, n, sb, [np.zeros(P * n, np.int32) for _ in range(P)]))
    try:
        O._replay(P, None, progs)
    except O._Stuck:
        return True
    except (ValueError, O._Crash):
        pass
    return False


def rooted_jobs():
    """gather_bine / scatter_bine / alltoall_bine (libbine_gather.c:16,
    libbine_scatter.c:14, libbine_alltoall.c:14 -- SURVEY.md section 2 row 7):
    N = elements per block; every root at P <= 8, a spread of roots at P = 16
    (the reference is correct at some, hangs, crashes or returns a wrong
    result at others: the fixtures pin which)"""
    sys.path.insert(0, ROOT)
    from oracle import oracle as O
    jobs = []
    for P in (1, 2, 3, 4, 5, 6, 7, 8, 16):
        for coll in ROOTED:
            roots = [0] if coll == "alltoall" else \
                list(range(P)) if P <= 8 else [0, 1, 2, 4, 5, 8, 9, 14, 15]
            for root in roots:
                if _replay_hangs(O, coll, P, root):
                    continue   # a deadlock: mpiexec would only time out (tests/test_oracle.py covers it)
                jobs.append((P, coll, "bine", "sum", 0, f"root{root}", ["float", "int64", "int8"], [1, 2, 7, 64, 333],
                             True))
    return jobs


def ops_jobs():
    """MPICH's logical and bitwise MPI_Ops through the reference's collectives
    (logical ops on sparsified inputs -- zeros, -0.0, NaN -- so that both truth
    values occur), and MAX / MIN on sparsified floats (NaN / signed-zero
    operand order through every schedule), plus the sparsified inputs
    themselves ("fill")"""
    jobs = [(8, "fill", "-", "sum", 0, "even_sparse", ALL_DT, [64], True)]
    for P in (1, 2, 4, 8):
        for op in LOGIC_OPS + BIT_OPS:
            rk, dts = ("even_sparse", LOGIC_DT) if op in LOGIC_OPS else ("even", BIT_DT)
            for a in ("bine_bdw_remap", "bine_bdw_static", "bine_lat", "ring"):
                jobs.append((P, "allreduce", a, op, 0, rk, dts, [13, 4096], True))
            for a in ("bine_permute_remap", "bine_static", "bine_block_by_block"):
                jobs.append((P, "reduce_scatter", a, op, 0, rk, dts, [P * 3, P * 1024], True))
            for a in ("bine_bdw", "bine_lat"):
                jobs.append((P, "reduce", a, op, 0, rk, dts, [13, 4096], True))
        for op in ("max", "min"):
            for a in ("bine_bdw_remap", "bine_lat", "rabenseifner"):
                jobs.append((P, "allreduce", a, op, 0, "even_sparse", ["float", "double"], [13, 4096], True))
            for a in ("bine_block_by_block", "bine_send_remap", "butterfly"):
                jobs.append((P, "reduce_scatter", a, op, 0, "even_sparse", ["float", "double"], [P * 3, P * 1024],
                             True))
            jobs.append((P, "reduce", "bine_lat", op, 0, "even_sparse", ["float"], [13, 4096], True))
        for op in ("maxloc", "minloc"):
            # MPI's pair types; the floating values sparsified (zeros, -0.0, NaN)
            for a in ("bine_bdw_remap", "bine_lat", "ring", "rabenseifner"):
                jobs.append((P, "allreduce", a, op, 0, "even_sparse", PAIR_DT, [13, 1000], True))
            for a in ("bine_permute_remap", "bine_block_by_block", "butterfly"):
                jobs.append((P, "reduce_scatter", a, op, 0, "even_sparse", PAIR_DT, [P * 3, P * 250], True))
            jobs.append((P, "reduce", "bine_bdw", op, 0, "even_sparse", PAIR_DT, [13, 1000], True))
        for op in ("sum", "prod"):
            # C99 complex (SUM / PROD only); plain and sparsified (zeros, -0.0) inputs
            for rk in ("even", "even_sparse"):
                for a in ("bine_bdw_remap", "bine_lat", "ring"):
                    jobs.append((P, "allreduce", a, op, 0, rk, CPLX_DT, [13, 1000], True))
                for a in ("bine_permute_remap", "bine_block_by_block"):
                    jobs.append((P, "reduce_scatter", a, op, 0, rk, CPLX_DT, [P * 3, P * 250], True))
                jobs.append((P, "reduce", "bine_bdw", op, 0, rk, CPLX_DT, [13, 1000], True))
    jobs.append((8, "fill", "-", "sum", 0, "even", PAIR_DT + CPLX_DT, [64], True))
    jobs.append((8, "fill", "-", "sum", 0, "even_sparse", PAIR_DT + CPLX_DT, [64], True))
    for P in (3, 6):
        for op in ("land", "bxor", "max"):
            rk, dts = ("even", ["int32"]) if op == "bxor" else ("even_sparse", ["float", "int8"])
            for a in ("ring", "bine_lat", "recursivedoubling"):
                jobs.append((P, "allreduce", a, op, 0, rk, dts, [13, 4096], True))
    return jobs


def odd_p_jobs():
    """P = 5 and 7 (prime, odd: neither power of two nor even) for every
    algorithm the reference runs at any P, both reduce-family collectives and
    the allgather family's any-P algorithms"""
    jobs = []
    for P in (5, 7):
        for a in ("ring", "rabenseifner", "recursivedoubling", "bine_lat", "bine_bdw_remap_segmented",
                  "bine_bdw_remap", "bine_bdw_static"):   # the last two: MPI_ERR_ARG
            seg = 64 if a == "bine_bdw_remap_segmented" else 0
            jobs.append((P, "allreduce", a, "sum", seg, "even", FEW_DT, [1, 7, 13, 333, 4096], True))
        for a in ("recursive_distance_doubling", "ring", "bine_send_remap", "bine_static", "butterfly"):
            jobs.append((P, "reduce_scatter", a, "sum", 0, "even", FEW_DT, [P, P * 5, P * 1000], True))
        for a in ("bine_lat", "bine_bdw"):
            jobs.append((P, "reduce", a, "sum", 0, "even", ["float"], [13], True))
    return jobs


def p16_jobs():
    """P = 16 (four Bine steps) for the reduce family's main algorithms"""
    jobs = []
    for a in ("bine_bdw_remap", "bine_bdw_static", "bine_lat", "bine_bdw_remap_segmented", "ring", "rabenseifner",
              "recursivedoubling", "bine_block_by_block_any_even"):
        seg = 64 if a == "bine_bdw_remap_segmented" else 0
        jobs.append((16, "allreduce", a, "sum", seg, "even", FEW_DT, [13, 4096, 65537], True))
    for a in RS_BINE + RS_CLASSIC:
        jobs.append((16, "reduce_scatter", a, "sum", 0, "even", FEW_DT, [16, 16 * 300], True))
    for a in ("bine_lat", "bine_bdw"):
        jobs.append((16, "reduce", a, "sum", 0, "even", FEW_DT, [13, 4096], True))
    return jobs


def large_p_jobs():
    """P = 32 and 64 (five and six Bine steps: beyond one node, the scale the
    reference's own campaigns run at) for the main algorithm of every family
    and the classic baselines"""
    jobs = []
    for P in (32, 64):
        for a in ("bine_bdw_remap", "bine_bdw_static", "bine_lat", "ring", "rabenseifner", "recursivedoubling"):
            jobs.append((P, "allreduce", a, "sum", 0, "even", FEW_DT, [13, 4099], True))
        jobs.append((P, "allreduce", "bine_bdw_remap_segmented", "sum", 64, "even", FEW_DT, [13, 4099], True))
        for a in ("bine_permute_remap", "bine_send_remap", "bine_static", "bine_block_by_block", "butterfly", "ring"):
            jobs.append((P, "reduce_scatter", a, "sum", 0, "even", FEW_DT, [P * 3, P * 100], True))
        for a in ("bine_bdw", "bine_lat"):
            jobs.append((P, "reduce", a, "sum", 0, "even", FEW_DT, [13, 4099], True))
        for a in ("bine_permute_remap", "bine_send_static", "bine_2_blocks", "k_bruck", "ring"):
            jobs.append((P, "allgather", a, "sum", 0, "even", FEW_DT, [3, 200], True))
        for a in ("bine_lat", "bine_bdw_remap", "bine_bdw_static", "scatter_allgather"):
            jobs.append((P, "bcast", a, "sum", 0, "even", FEW_DT, [7, P + 1, 4099], True))
        jobs.append((P, "bcast", "bine_lat_new", "sum", 0, f"root{P - 1}", FEW_DT, [7, 4099], True))
        for coll in ROOTED:
            jobs.append((P, coll, "bine", "sum", 0, "root0", FEW_DT, [1, 33], True))
    # the operators' semantics through deeper trees: P = 16 and 32
    for P in (16, 32):
        for op, rk, dts in (("max", "even_sparse", ["float", "double"]), ("min", "even_sparse", ["float"]),
                            ("prod", "even", ["float", "int32"]), ("land", "even_sparse", ["float", "int8"]),
                            ("bxor", "even", ["int64", "int16"]), ("maxloc", "even_sparse", PAIR_DT),
                            ("minloc", "even_sparse", PAIR_DT)):
            for a in ("bine_bdw_remap", "bine_lat"):
                jobs.append((P, "allreduce", a, op, 0, rk, dts, [13, 1000], True))
            jobs.append((P, "reduce_scatter", "bine_permute_remap", op, 0, rk, dts, [P * 3, P * 64], True))
            jobs.append((P, "reduce", "bine_bdw", op, 0, rk, dts, [13, 1000], True))
    # the allgather family with MPI_IN_PLACE (the own block already in rbuf)
    for P in (1, 2, 3, 4, 8):
        for a in AG_ALGOS:
            jobs.append((P, "allgather", a, "sum", 0, "even_inplace", ["float", "int64"], [7, 333], True))
    # MPI_IN_PLACE and ragged blocks through P = 16's four steps
    for a in AR_BINE + AR_CLASSIC:
        jobs.append((16, "allreduce", a, "sum", 0, "even_inplace", FEW_DT, [13, 4099], True))
    for a in RS_BINE + RS_CLASSIC:
        jobs.append((16, "reduce_scatter", a, "sum", 0, "even_inplace", FEW_DT, [16 * 3, 16 * 100], True))
        if a in RS_RAGGED_OK:
            jobs.append((16, "reduce_scatter", a, "sum", 0, "ragged", FEW_DT, [16 * 4, 16 * 50], True))
    for a in ("bine_lat", "bine_bdw"):
        jobs.append((16, "reduce", a, "sum", 0, "even_inplace", FEW_DT, [13, 4099], True))
    # non-power-of-two sizes past 8 for the algorithms that run at any P (the
    # others' error returns / refusals are pinned at P = 3, 5, 6, 7)
    for P in (12, 24):
        for a in ("ring", "rabenseifner", "bine_lat", "recursivedoubling"):
            jobs.append((P, "allreduce", a, "sum", 0, "even", FEW_DT, [13, 4099], True))
        jobs.append((P, "allreduce", "bine_bdw_remap_segmented", "sum", 64, "even", FEW_DT, [13, 4099], True))
        for a in ("ring", "butterfly", "recursivehalving", "bine_send_remap"):
            jobs.append((P, "reduce_scatter", a, "sum", 0, "even", FEW_DT, [P * 3, P * 100], True))
        for a in ("ring", "k_bruck", "sparbit"):
            jobs.append((P, "allgather", a, "sum", 0, "even", FEW_DT, [3, 200], True))
        jobs.append((P, "bcast", "scatter_allgather", "sum", 0, "even", FEW_DT, [7, P + 1, 4099], True))
    return jobs


def inplace_jobs():
    """MPI_IN_PLACE through every reduce-family algorithm (the reference's own
    in-place code paths, e.g. libbine_allreduce.c:849-852,
    libbine_reduce_scatter.c:810-813)"""
    jobs = []
    for P in (1, 2, 4, 8):
        for a in AR_BINE + AR_CLASSIC + ["bine_bdw_remap_segmented"]:
            seg = 64 if a == "bine_bdw_remap_segmented" else 0
            jobs.append((P, "allreduce", a, "sum", seg, "even_inplace", FEW_DT, [13, 4096], True))
        for a in RS_BINE + RS_CLASSIC:
            jobs.append((P, "reduce_scatter", a, "sum", 0, "even_inplace", FEW_DT, [P * 3, P * 1024], True))
        for a in ("bine_lat", "bine_bdw"):
            jobs.append((P, "reduce", a, "sum", 0, "even_inplace", FEW_DT, [13, 4096], True))
    return jobs


def _is_odd_p_case(c):
    return c["P"] in (5, 7) and c["coll"] != "allgather"


def _is_ops_case(c):
    return c["op"] in LOGIC_OPS + BIT_OPS + ["maxloc", "minloc"] or c["rcounts"].endswith("_sparse") or \
        c["dtype"] in ("float_int", "double_int", "long_int", "2int", "short_int") + tuple(CPLX_DT)


def main():
    if not os.path.exists(BIN):
        sys.exit("build the reference first: make -C oracle ref")
    os.makedirs(OUT, exist_ok=True)
    only = sys.argv[sys.argv.index("--only") + 1] if "--only" in sys.argv else None
    if only:
        # regenerate one collective's cases, keep everything else as it is
        old, prev = load_fixtures()
        if only == "inplace":
            index = [c for c in old if not c["rcounts"].endswith("_inplace")]
            keep = {c["id"] for c in index}
            arrays = {k: v for k, v in prev.items() if k in keep}
            return capture(inplace_jobs(), index, arrays)
        if only == "p16":
            index = [c for c in old if not (c["P"] == 16 and c["coll"] != "allgather")]
            keep = {c["id"] for c in index}
            arrays = {k: v for k, v in prev.items() if k in keep}
            return capture(p16_jobs(), index, arrays)
        if only == "oddp":
            index = [c for c in old if not _is_odd_p_case(c)]
            keep = {c["id"] for c in index}
            arrays = {k: v for k, v in prev.items() if k in keep}
            return capture(odd_p_jobs(), index, arrays)
        if only == "ops":
            index = [c for c in old if not _is_ops_case(c)]
            keep = {c["id"] for c in index}
            arrays = {k: v for k, v in prev.items() if k in keep}
            return capture(ops_jobs(), index, arrays)
        if only == "bcast_bdw":
            index = [c for c in old if not (c["coll"] == "bcast" and c["algo"] in BC_BDW)]
            keep = {c["id"] for c in index}
            arrays = {k: v for k, v in prev.items() if k in keep}
            return capture(bcast_bdw_jobs(), index, arrays)
        if only == "largep":
            index = [c for c in old if c["P"] not in (12, 24, 32, 64) and
                     not (c["P"] == 16 and (c["op"] != "sum" or c["rcounts"] in ("even_inplace", "ragged"))) and
                     not (c["coll"] == "allgather" and c["rcounts"] == "even_inplace")]
            keep = {c["id"] for c in index}
            arrays = {k: v for k, v in prev.items() if k in keep}
            return capture(large_p_jobs(), index, arrays)
        if only == "rooted":
            index = [c for c in old if c["coll"] not in ROOTED]
            keep = {c["id"] for c in index}
            arrays = {k: v for k, v in prev.items() if k in keep}
            return capture(rooted_jobs(), index, arrays)
        index = [c for c in old if c["coll"] != only]
        arrays = {k: v for k, v in prev.items() if not k.startswith(only + ".")}
        jobs = {"allgather": allgather_jobs, "bcast": bcast_jobs}[only]()
        return capture(jobs, index, arrays)
    jobs = []  # (P, coll, algo, op, segsize, rk, dtypes, ns, store_small)
    # input generator pin
    jobs.append((8, "fill", "-", "sum", 0, "even", ALL_DT, [64], True))
    for P in (1, 2, 4, 8):
        for a in AR_BINE:
            jobs.append((P, "allreduce", a, "sum", 0, "even", ALL_DT, SMALL_N + MID_N, True))
        for seg in (0, 16, 64, 4096):
            jobs.append((P, "allreduce", "bine_bdw_remap_segmented", "sum", seg, "even",
                         ["float", "int64", "int8"], SMALL_N + MID_N, True))
        for a in AR_CLASSIC:
            jobs.append((P, "allreduce", a, "sum", 0, "even", FEW_DT, SMALL_N + MID_N, True))
        for a in RS_BINE + RS_CLASSIC:
            dts = ALL_DT if a in RS_BINE else FEW_DT
            jobs.append((P, "reduce_scatter", a, "sum", 0, "even", dts, [P * k for k in (1, 3, 16)] + [P * 8192 + 0], True))
            if a in RS_RAGGED_OK and P > 1:
                jobs.append((P, "reduce_scatter", a, "sum", 0, "ragged", FEW_DT, [P * 4, P * 50], True))
        for a in ("bine_lat", "bine_bdw"):
            jobs.append((P, "reduce", a, "sum", 0, "even", ALL_DT, SMALL_N + MID_N, True))
        for op in ("max", "min", "prod"):
            jobs.append((P, "allreduce", "bine_bdw_remap", op, 0, "even", ["float", "double", "int32"], [13, 4096], True))
            jobs.append((P, "reduce_scatter", "bine_permute_remap", op, 0, "even", ["float", "int32"], [P * 3, P * 1024], True))
            jobs.append((P, "reduce", "bine_bdw", op, 0, "even", ["float", "int32"], [13, 4096], True))
    for P in (3, 6):
        for a in sorted(AR_NONPOW2):
            seg = 64 if a == "bine_bdw_remap_segmented" else 0
            jobs.append((P, "allreduce", a, "sum", seg, "even", FEW_DT, [1, 7, 13, 333, 4096], True))
        for a in sorted(RS_NONPOW2):
            jobs.append((P, "reduce_scatter", a, "sum", 0, "even", FEW_DT, [P, P * 5, P * 1000], True))
        for a in ("bine_lat", "bine_bdw"):
            jobs.append((P, "reduce", a, "sum", 0, "even", ["float"], [13], True))
    # large: digests only (the headline schedule at a non-power-of-two-friendly size)
    for a, seg in (("bine_bdw_remap", 0), ("bine_bdw_static", 0), ("bine_bdw_remap_segmented", 65536),
                   ("bine_bdw_remap_segmented", 0)):
        jobs.append((8, "allreduce", a, "sum", seg, "even", ["float"], [1000003], False))
    jobs.append((8, "reduce_scatter", "bine_permute_remap", "sum", 0, "even", ["float"], [8 * 131072 + 8 * 3], False))
    jobs.append((8, "allreduce", "bine_bdw_remap", "sum", 0, "even", ["double", "int64"], [262147], False))
    jobs += allgather_jobs()
    jobs += ops_jobs()
    jobs += odd_p_jobs()
    jobs += p16_jobs()
    jobs += inplace_jobs()
    jobs += bcast_jobs()
    jobs += bcast_bdw_jobs()
    jobs += rooted_jobs()
    jobs += large_p_jobs()
    capture(jobs, [], {})


def capture(jobs, index, arrays):
    for (P, coll, algo, op, seg, rk, dts, ns, store) in jobs:
        # the reference hangs on some shapes (e.g. odd P in the any_even
        # variants): a short limit, then the cases are re-run one by one
        short = coll in ("allgather", "bcast")
        # the rooted collectives' fixtures are tiny: a hang shows within seconds
        recs = run_case(P, coll, algo, op, seg, rk, dts, ns, timeout=15 if coll in ROOTED else 60 if short else 120)
        if any(r[2] is None for r in recs):
            # one crashing case (e.g. the static variant's tmp_buf overflow,
            # libbine_allreduce.c:724 vs :749-765) kills the whole mpiexec:
            # re-run the missing cases one at a time
            fixed = []
            for rec in recs:
                if rec[2] is None:
                    rec = run_case(P, coll, algo, op, seg, rk, [rec[0]], [rec[1]],
                                   timeout=5 if coll in ROOTED else 20 if short else 120)[0]
                fixed.append(rec)
            recs = fixed
        for dt, n, rets, outs, failed in recs:
            cid = f"{coll}.{algo}.{op}.{dt}.P{P}.N{n}.seg{seg}.{rk}"
            rec = {"id": cid, "coll": coll, "algo": algo, "op": op, "dtype": dt, "P": P, "N": n,
                   "segsize": seg, "rcounts": rk, "seed_base": SEED}
            if rets is None:
                rec["status"] = "no_output"  # reference aborted / hung
            else:
                rec["status"] = "ok"
                rec["rets"] = rets
                rec["outn"] = [len(o) // ESZ[dt] for o in outs]
                rec["sha256"] = [hashlib.sha256(o).hexdigest() for o in outs]
                # identical outputs on every rank (allreduce) are stored once
                same = len(set(rec["sha256"])) == 1
                blob = outs[0] if same else b"".join(outs)
                small = store and len(blob) <= 16 * 1024
                if small:
                    arrays[cid] = np.frombuffer(blob, dtype=np.uint8)
                rec["stored"] = ("rank0" if same else "all") if small else None
            index.append(rec)
        print(f"P={P} {coll} {algo} {op} seg={seg} {rk}: {len(recs)} cases", flush=True)
    write_fixtures(index, arrays)


def write_fixtures(index, arrays):
    """tests/golden/index.json.gz + outputs.npz.  Stored outputs are kept once
    per distinct content (many algorithms, in- and out-of-place runs give the
    same bytes): npz members are named by a content hash, and each stored case
    names its member in "blob"."""
    blobs = {}
    for rec in index:
        a = arrays.get(rec["id"])
        if a is None:
            continue
        name = "b" + hashlib.sha256(a.tobytes()).hexdigest()[:24]
        blobs[name] = a
        rec["blob"] = name
    doc = {"generator": "tools/make_golden.py", "reference": "HLC-Lab/pico libbine @ 2025-07-25",
           "mpi": "MPICH 3.3.2 (ch3:nemesis)", "cases": index}
    with gzip.GzipFile(os.path.join(OUT, "index.json.gz"), "wb", mtime=0) as f:
        f.write(json.dumps(doc, separators=(",", ":")).encode())
    np.savez_compressed(os.path.join(OUT, "outputs.npz"), **blobs)
    print(len(index), "cases,", len(arrays), "stored,", len(blobs), "distinct")


def load_fixtures():
    """(index, {case id: stored bytes}) of the committed fixtures"""
    with gzip.open(os.path.join(OUT, "index.json.gz"), "rt") as f:
        index = json.load(f)["cases"]
    npz = np.load(os.path.join(OUT, "outputs.npz"), allow_pickle=False)
    arrays = {c["id"]: npz[c["blob"]] for c in index if c.get("blob")}
    return index, arrays


if __name__ == "__main__":
    main()
