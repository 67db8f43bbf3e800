"""Randomized parity sweep of the device path (fixed seeds, so every run checks
the same cases): collective x algorithm x P x count x element type x operator x
transport setting (relay, flat allgather / reduce-scatter phases, pipelining
chunk, multi-tree mode on integer types) x in place, on loopback ranks, bit-exact against the oracle (the CPU
restatement pinned by the reference's vectors, tests/test_oracle.py).  Where
the oracle reports an error (the reference's MPI_ERR_ARG / MPI_ERR_SIZE, or a
reference assert / hang) the device path must return an error too.  The oracle itself
reports MPI_ERR_ARG where the reference hangs or overruns (the remap and
block-by-block reduce-scatters at non-power-of-two P), as the device path does."""
import random

import numpy as np
import pytest

import pico_amd  # noqa: E402  (after torch, via test_gpu)
from oracle import oracle as O
from test_gpu import STATUS_OF_MPI, comms, oracle_bcast, run_loopback, sha

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

INTS = ["int8", "uint8", "int16", "uint16", "int32", "uint32", "int64", "uint64"]
PLAIN = INTS + ["float", "double"]
OPS_OF = {
    **{d: ["sum", "prod", "max", "min", "land", "lor", "lxor", "band", "bor", "bxor"] for d in PLAIN},
    "float": ["sum", "prod", "max", "min", "land", "lor", "lxor"],
    "double": ["sum", "prod", "max", "min", "land", "lor", "lxor"],
    "float_int": ["maxloc", "minloc"], "double_int": ["maxloc", "minloc"], "2int": ["maxloc", "minloc"],
    "c_float_complex": ["sum", "prod"], "c_double_complex": ["sum", "prod"],
}
COLLS = {"allreduce": list(pico_amd.ALGOS["allreduce"]), "reduce_scatter": list(pico_amd.ALGOS["reduce_scatter"]),
         "reduce": list(pico_amd.ALGOS["reduce"]), "allgather": list(pico_amd.ALGOS["allgather"]),
         "bcast": list(pico_amd.ALGOS["bcast"])}


def _case(rng):
    coll = rng.choice(["allreduce"] * 3 + ["reduce_scatter"] * 2 + ["reduce", "allgather"])
    algo = rng.choice(COLLS[coll])
    P = rng.choice([1, 2, 3, 4, 4, 5, 6, 8, 8, 16])
    dt = rng.choice(list(OPS_OF))
    op = rng.choice(OPS_OF[dt])
    n = rng.choice([1, 2, 7, 64, 333, 1000, 4097, rng.randint(1, 30000)])
    opts = {"relay": rng.choice([0, 0, 64, 4096]), "flat_ag": rng.random() < 0.4, "flat_rs": rng.random() < 0.4,
            "chunk": rng.choice([0, 0, 256, 4096, 65536]), "in_place": rng.random() < 0.25,
            "sparse": rng.random() < 0.5, "ragged": rng.random() < 0.5, "trees": rng.random() < 0.25}
    return coll, algo, P, dt, op, n, opts


def expected_status(rets):
    """the device statuses the oracle's returns map to: MPI_ERR_ARG / _SIZE /
    _ROOT -> BINE_ERR_ARG / _SIZE / _ROOT; where the reference asserts or hangs
    (the oracle's ASSERT / DEADLOCK) the device path reports BINE_ERR_ARG
    (DESIGN.md deviations)"""
    return [0 if r == 0 else STATUS_OF_MPI.get(r, 1) for r in rets]


def rng_root(P, n):
    return (n * 7 + 3) % P   # deterministic from the case: 0 for about 1 in P cases


def _run(coll, algo, P, dt, op, n, o):
    mk = (lambda r: O.sparsify(O.fill(dt, m, 99 + r), dt, r)) if o["sparse"] else (lambda r: O.fill(dt, m, 99 + r))
    rk = None
    if coll == "reduce_scatter":
        rk = [n // P + ((i % 3) if o["ragged"] and algo != "bine_permute_remap" else 0) for i in range(P)]
        m = sum(rk)
    else:
        m = n
    sb = [mk(r) for r in range(P)]
    if coll == "bcast":   # pure data movement, in place; any root (the root-0-only trees: ERR_ROOT elsewhere)
        root = rng_root(P, n)
        want, rets = oracle_bcast(algo, sb, dt, root)
        for c in comms(P):
            c.set_flat_ag(o["flat_ag"])
        outs, st = run_loopback(coll, algo, sb, dt, root=root, relay=o["relay"])
        return want, rets, outs, st
    if coll == "allgather":   # pure data movement: any type, no operator, out of place
        want, rets = O.allgather(algo, sb, dt)
        if algo == "recursivedoubling" and P & (P - 1):
            rets = [O.ERR_ARG] * P   # the reference gathers nothing and reports success; here MPI_ERR_ARG
        if algo == "bine_block_by_block_any_even" and P % 2:
            rets = [O.ERR_ARG] * P   # odd P (1 included) hangs / crashes in the reference (no vector); MPI_ERR_ARG here
        for c in comms(P):
            c.set_flat_ag(o["flat_ag"])
        outs, st = run_loopback(coll, algo, sb, dt, relay=o["relay"])
        return want, rets, outs, st
    if coll == "allreduce":
        want, rets = O.allreduce(algo, sb, dt, op, 64 if algo == "bine_bdw_remap_segmented" else 0)
    elif coll == "reduce_scatter":
        want, rets = O.reduce_scatter(algo, sb, rk, dt, op)
        if P == 1 and algo in ("butterfly", "bine_block_by_block"):
            want = [sb[0][: rk[0]]]   # the P = 1 copy the reference omits (DESIGN.md deviations)
    else:
        w, rets = O.reduce(algo, sb, dt, op)
        want = [w]
    # multi-tree mode (P = 4, 8) relabels ranks: bit-exact vs the reference's
    # schedule only where the operator is associative and commutative in the
    # element type -- the integer types
    trees = o["trees"] and dt in INTS and P in (4, 8)
    for c in comms(P):
        c.set_flat_ag(o["flat_ag"])
        c.set_flat_rs(o["flat_rs"])
        c.set_chunk(o["chunk"])
        c.set_trees(trees)
    outs, st = run_loopback(coll, algo, sb, dt, op, rk, 64 if algo == "bine_bdw_remap_segmented" else 0,
                            in_place=o["in_place"], relay=o["relay"])
    return want, rets, outs, st


@pytest.mark.parametrize("seed", range(20))
def test_random_configurations_bit_exact(dev_fuzz, seed):
    rng = random.Random(1000 + seed)
    bad = []
    try:
        for _ in range(60):
            coll, algo, P, dt, op, n, o = _case(rng)
            want, rets, outs, st = _run(coll, algo, P, dt, op, n, o)
            if any(rets):
                if list(st) != expected_status(rets):
                    bad.append((coll, algo, P, dt, op, n, o, "expected these errors", rets, st))
                continue
            if any(st):
                bad.append((coll, algo, P, dt, op, n, o, "status", st))
            elif any(sha(x) != sha(w) for x, w in zip(outs, want)):
                bad.append((coll, algo, P, dt, op, n, o, "data"))
    finally:
        for P in (1, 2, 3, 4, 5, 6, 8, 16):
            for c in comms(P):
                c.set_relay(0)
                c.set_flat_ag(False)
                c.set_flat_rs(False)
                c.set_chunk(0)
                c.set_trees(False)
    assert not bad, bad[:6]


@pytest.mark.parametrize("seed", range(4))
def test_random_bcast_bit_exact(dev_fuzz, seed):
    """bcast, latency trees and (round 5) the bandwidth algorithms: random P
    (non-powers of two: MPI_ERR_SIZE where the reference says so), root
    (root-0-only trees: MPI_ERR_ROOT elsewhere), type, count (below P:
    MPI_ERR_COUNT for the bandwidth ones), relay, vs the oracle's
    message-level replay (tests/test_oracle.py pins it)"""
    rng = random.Random(5000 + seed)
    bad = []
    try:
        for _ in range(40):
            algo = rng.choice(COLLS["bcast"])
            P = rng.choice([1, 2, 3, 4, 4, 6, 8, 8, 16])
            dt = rng.choice(list(OPS_OF))
            n = rng.choice([1, 2, 7, 64, 333, 1000, 4097, rng.randint(1, 30000)])
            o = {"relay": rng.choice([0, 0, 64, 4096]), "flat_ag": rng.random() < 0.4, "sparse": rng.random() < 0.5}
            want, rets, outs, st = _run("bcast", algo, P, dt, "sum", n, o)
            if any(rets):
                if list(st) != expected_status(rets):
                    bad.append((algo, P, dt, n, o, "expected these errors", rets, st))
            elif any(st):
                bad.append((algo, P, dt, n, o, "status", st))
            elif any(sha(x) != sha(w) for x, w in zip(outs, want)):
                bad.append((algo, P, dt, n, o, "data"))
    finally:
        for P in (1, 2, 3, 4, 6, 8, 16):
            for c in comms(P):
                c.set_relay(0)
                c.set_flat_ag(False)
    assert not bad, bad[:6]


@pytest.mark.parametrize("seed", range(3))
def test_random_rooted_bit_exact(dev_fuzz, seed):
    """gather / scatter / alltoall (round 5): random P, root, type, block size,
    direct form, relay, vs the collective where the reference delivers it and
    the refusal elsewhere (tests/rooted_util.py; tests/test_oracle.py pins the
    replay that decides)"""
    import rooted_util as R
    rng = random.Random(7000 + seed)
    bad = []
    try:
        for _ in range(30):
            coll = rng.choice(R.ROOTED)
            P = rng.choice([1, 2, 3, 4, 4, 6, 8, 8, 16])
            root = 0 if coll == "alltoall" else rng.choice([0, 0, rng.randrange(P)])
            dt = rng.choice(list(OPS_OF))
            n = rng.choice([1, 2, 7, 64, 333, 1000, 4097, rng.randint(1, 20000)])
            flat, relay = rng.random() < 0.4, rng.choice([0, 0, 64, 4096])
            sb = R.inputs(coll, dt, n, P, seed_base=31 + seed)
            want, exp = R.expect(coll, sb, dt, root, P, n)
            for c in comms(P):
                c.set_flat_ag(flat)
            outs, st = run_loopback(coll, "bine", sb, dt, root=root, relay=relay)
            if list(st) != [exp] * P:
                bad.append((coll, P, root, dt, n, flat, relay, "status", st, exp))
            elif not exp and any(O.canonical(o) != (b"" if w is None else O.canonical(w)) for o, w in zip(outs, want)):
                bad.append((coll, P, root, dt, n, flat, relay, "data"))
    finally:
        for P in (1, 2, 3, 4, 6, 8, 16):
            for c in comms(P):
                c.set_relay(0)
                c.set_flat_ag(False)
    assert not bad, bad[:6]


@pytest.fixture(scope="module")
def dev_fuzz():
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    np.seterr(all="ignore")
    return torch.device("cuda:0")
