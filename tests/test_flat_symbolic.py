"""The flat phases compute the literal schedule's EXPRESSIONS, not just its
numbers: both plans run through the rendezvous simulator (tests/plan_sim.py)
on symbolic elements -- input element i of rank r is the leaf ("x", r, i) and
every MPI_Reduce_local(in, inout) builds the node ("op", inout, in) -- and the
results must be the identical expression trees, element for element: same
operands, same association, same operand order.  The literal plans are the
ones pinned bit-for-bit against the reference's golden vectors
(tests/test_oracle.py, tests/test_plan.py), so this proves the flat
reduce-scatter / flat allgather forms (REDUCE_TREE) reproduce the reference
for every dtype and operator, NaN payloads and signed zeros included."""
import contextlib

import numpy as np
import pytest

import plan_sim
from oracle import oracle as O


@contextlib.contextmanager
def symbolic():
    def sym_reduce(inp, inout, dtype, op="sum"):
        for k in range(inout.size):
            inout[k] = ("op", inout[k], inp[k])
    saved = O.reduce_local
    O.NP_DTYPES["sym"] = object
    O.reduce_local = sym_reduce
    try:
        yield
    finally:
        O.reduce_local = saved
        del O.NP_DTYPES["sym"]


def leaves(P, n):
    out = []
    for r in range(P):
        a = np.empty(n, dtype=object)
        for i in range(n):
            a[i] = ("x", r, i)
        out.append(a)
    return out


CASES = [("allreduce", "bine_bdw_remap"), ("allreduce", "bine_bdw_static"),
         ("allreduce", "bine_bdw_remap_segmented"), ("allreduce", "rabenseifner"), ("allreduce", "bine_lat"),
         ("reduce_scatter", "bine_permute_remap"), ("reduce_scatter", "bine_send_remap"),
         ("reduce_scatter", "bine_static"), ("reduce_scatter", "bine_block_by_block"),
         ("reduce_scatter", "recursivehalving"), ("reduce", "bine_bdw"), ("reduce", "bine_lat"),
         ("allreduce", "recursivedoubling"), ("reduce_scatter", "recursive_distance_doubling"),
         ("reduce_scatter", "butterfly"), ("allreduce", "bine_block_by_block_any_even"),
         ("reduce_scatter", "bine_block_by_block_any_even"), ("allreduce", "ring"), ("reduce_scatter", "ring")]


@pytest.mark.parametrize("coll,algo", CASES)
@pytest.mark.parametrize("P", [2, 4, 8, 16])
def test_flat_plans_build_the_literal_expressions(coll, algo, P):
    with symbolic():
        for n, in_place in ((3 * P + 5, False), (2 * P + 1, True)):
            rc = None
            if coll == "reduce_scatter":
                rc = [3] * P if algo == "bine_permute_remap" else [2 + (i % 3) for i in range(P)]
            sb = leaves(P, sum(rc) if rc else n)
            kw = dict(rcounts=rc, segsize=64 * 8, in_place=in_place)
            literal = plan_sim.run(coll, algo, [x.copy() for x in sb], "sym", **kw)
            flat = plan_sim.run(coll, algo, [x.copy() for x in sb], "sym", chunk_bytes=16, flat_rs=True,
                                flat_ag=True, **kw)
            ranks = [0] if coll == "reduce" else range(P)
            for r in ranks:
                assert list(flat[r]) == list(literal[r]), (coll, algo, P, in_place, r)
            # and the flat schedule really is the flat one: one all-peers exchange, then a
            # REDUCE_TREE (the rings: their chain folded by pairwise reductions)
            prims, _ = plan_sim.scheduled_prims(coll, algo, P, 0, 16, flat_rs=True, flat_ag=True,
                                                count=n, rcounts=rc, esz=8, segsize=64 * 8, in_place=in_place)
            if algo == "ring":
                assert not any(p["type"] == "REDUCE_TREE" for p in prims)
                first = [p for p in prims if p["group"] == min(q["group"] for q in prims if q["type"] == "SEND")]
                assert {p["peer"] for p in first if p["type"] == "SEND"} == set(range(1, P)) or P == 1
            else:
                assert any(p["type"] == "REDUCE_TREE" for p in prims)
                assert not any(p["type"] in ("REDUCE", "REDUCE3") for p in prims)


def test_symbolic_check_sees_operand_order():
    """negative control: the same flat schedule with block_by_block's swapped
    top level un-swapped builds different expressions (operand order only)"""
    orig = plan_sim.scheduled_prims

    def unswapped(*a, **k):
        prims, info = orig(*a, **k)
        for p in prims:
            if p["type"] == "REDUCE_TREE":
                p["flags"] &= 0xFF
        return prims, info
    with symbolic():
        rc = [3] * 4
        sb = leaves(4, 12)
        lit = plan_sim.run("reduce_scatter", "bine_block_by_block", [x.copy() for x in sb], "sym", rcounts=rc)
        plan_sim.scheduled_prims = unswapped
        try:
            bad = plan_sim.run("reduce_scatter", "bine_block_by_block", [x.copy() for x in sb], "sym", rcounts=rc,
                               chunk_bytes=16, flat_rs=True)
        finally:
            plan_sim.scheduled_prims = orig
        assert not all(list(a) == list(b) for a, b in zip(lit, bad))
