"""gather_bine / scatter_bine / alltoall_bine (libbine_gather.c:16-96,
libbine_scatter.c:14-151, libbine_alltoall.c:14-147; SURVEY.md section 2
row 7, widening past section 8): the planner's per-rank plans, run for every
rank by the host rendezvous simulator (tests/plan_sim.py), against the
oracle's message-level replay of the reference (itself pinned by the
reference's own outputs in tests/golden, tests/test_oracle.py):

* where the reference delivers the collective, the literal plan and the
  direct form (flat_ag) deliver the same bytes;
* everywhere else -- non-power-of-two P, odd roots, some even scatter roots,
  where the reference hangs, aborts, reads past its buffers or returns
  something else -- the plan is refused with BINE_ERR_ROOT (power-of-two P)
  or BINE_ERR_SIZE, and MPI_IN_PLACE with BINE_ERR_ARG;
* the literal plans keep the reference's message pattern (a tree for
  gather / scatter, log2 P pairwise exchanges for alltoall)."""
import numpy as np
import pytest

import golden_util as G
import pico_amd
import plan_sim
import rooted_util as R
from oracle import oracle as O


def _roots(coll, P):
    if coll == "alltoall":
        return [0]
    return list(range(P)) if P <= 8 else [0, 1, 2, 4, 5, 8, 9, 14, 15]


@pytest.mark.parametrize("P", [1, 2, 3, 4, 5, 6, 7, 8, 16])
@pytest.mark.parametrize("coll", R.ROOTED)
def test_plans_deliver_or_refuse(coll, P):
    for root in _roots(coll, P):
        for dt, n in (("int32", 3), ("int8", 1)):
            sb = R.inputs(coll, dt, n, P)
            want, st = R.expect(coll, sb, dt, root, P, n)
            ins = [s if (coll != "scatter" or r == root) else None for r, s in enumerate(sb)]
            for flat in (False, True):
                if st:
                    with pytest.raises(pico_amd.BineError) as e:
                        plan_sim.run(coll, "bine", ins, dt, root=root, chunk_bytes=1 << 20, flat_ag=flat)
                    assert e.value.status == st, (coll, P, root)
                    continue
                got = plan_sim.run(coll, "bine", ins, dt, root=root, chunk_bytes=1 << 20, flat_ag=flat)
                for r in range(P):
                    w = b"" if want[r] is None else O.canonical(want[r])
                    assert O.canonical(got[r]) == w, (coll, P, root, r, flat)


def test_supported_roots():
    """the (P, root) pairs the product accepts: every power-of-two P at root 0
    (pico_core's root, pico_core_utils.c:505-547) and at the even roots where
    the reference delivers the collective"""
    def ok(coll, P, root):
        try:
            pico_amd.plan(coll, "bine", P, 0, count=4, root=root, esz=4)
            return True
        except pico_amd.BineError:
            return False
    for P in (1, 2, 4, 8, 16, 32):
        for coll in R.ROOTED:
            assert ok(coll, P, 0), (coll, P)
    assert [r for r in range(8) if ok("gather", 8, r)] == [0, 2, 4, 6]
    assert [r for r in range(8) if ok("scatter", 8, r)] == [0, 2, 4, 6]
    assert [r for r in range(16) if ok("scatter", 16, r)] == [0, 2, 4, 6, 10, 12, 14]
    for P in (3, 5, 6, 7, 12):
        assert not any(ok(c, P, 0) for c in R.ROOTED), P


def test_errors():
    for coll in R.ROOTED:
        with pytest.raises(pico_amd.BineError) as e:
            pico_amd.plan(coll, "bine", 4, 0, count=4, root=0, esz=4, in_place=True)
        assert e.value.status == 1   # MPI_IN_PLACE: the reference memcpy's from it
    for coll in ("gather", "scatter"):
        for root in (-1, 4):
            with pytest.raises(pico_amd.BineError) as e:
                pico_amd.plan(coll, "bine", 4, 0, count=4, root=root, esz=4)
            assert e.value.status == 8


@pytest.mark.parametrize("P", [2, 4, 8, 16])
def test_message_pattern(P):
    n = 5
    # gather / scatter at root 0: a tree -- every non-root sends (gather) or
    # receives (scatter) its subtree once; P - 1 + wrapped messages in all
    for coll, kind in (("gather", "SEND"), ("scatter", "RECV")):
        per = []
        for r in range(P):
            prims, tmp = pico_amd.plan(coll, "bine", P, r, count=n, root=0, esz=4)
            xs = [p for p in prims if p["type"] == kind]
            per.append(len({p["group"] for p in xs}) if r else len(xs))
            assert all(p["count"] % n == 0 for p in prims)
        assert per[0] == 0 and all(1 <= k <= 2 for k in per[1:]), (coll, per)
    # alltoall: log2 P exchanges of P / 2 blocks with the negabinary partner
    for r in range(P):
        prims, tmp = pico_amd.plan("alltoall", "bine", P, r, count=n, esz=4)
        xs = [p for p in prims if p["type"] in ("SEND", "RECV")]
        assert len(xs) == 2 * (P.bit_length() - 1)
        assert all(p["count"] == P // 2 * n for p in xs)
        assert tmp[0] == P * n


def test_flat_forms_are_one_exchange():
    P, n = 8, 7
    for coll in R.ROOTED:
        for r in range(P):
            ops, _, _, info = pico_amd.schedule(coll, "bine", P, r, count=n, root=0, esz=4, chunk_bytes=1 << 20,
                                                info=True, flat_ag=True)
            xs = [o for o in ops if any(p["type"] in ("SEND", "RECV") for p in o["prims"])]
            assert len(xs) == 1, (coll, r)


@pytest.mark.parametrize("coll", R.ROOTED)
def test_plans_reproduce_reference_goldens(coll):
    """the captured reference outputs, wherever the product accepts the call"""
    n_ok = 0
    for c in G.select(coll=coll):
        P, N, dt, root = c["P"], c["N"], c["dtype"], G.root(c)
        sb = R.inputs(coll, dt, N, P, c["seed_base"])
        want, st = R.expect(coll, sb, dt, root, P, N)
        if st:
            continue
        ins = [s if (coll != "scatter" or r == root) else None for r, s in enumerate(sb)]
        got = plan_sim.run(coll, "bine", ins, dt, root=root, chunk_bytes=1 << 20)
        if c["status"] != "ok":
            assert coll == "scatter" and P == 1, c["id"]   # the deviation
            continue
        assert not any(c["rets"]), c["id"]
        assert G.check_rank_outputs(c, got) == [], c["id"]
        n_ok += 1
    assert n_ok >= 60
