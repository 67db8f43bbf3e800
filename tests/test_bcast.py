"""bcast latency trees (libbine_bcast.c:189-452, widening past SURVEY.md §8):
the planner's per-rank plans, run by the host rendezvous simulator
(tests/plan_sim.py), deliver the root's buffer to every rank, deadlock-free,
with the reference's message pattern: every non-root rank receives the whole
buffer exactly once, from its tree parent, and log2(P) steps in all.  The
reference's error returns: MPI_ERR_SIZE at non-power-of-two P, MPI_ERR_ROOT
for bcast_bine_lat / _reversed at root != 0 (:198-210, :290-302, :381, :417)."""
import numpy as np
import pytest

import pico_amd
import plan_sim
from oracle import oracle as O

BC = list(pico_amd.ALGOS["bcast"])
BC_LAT = [a for a in BC if a not in O.BC_BDW]   # the latency trees: whole-buffer messages


@pytest.mark.parametrize("P", [1, 2, 4, 8, 16])
@pytest.mark.parametrize("algo", BC_LAT)
def test_bcast_delivers_root_buffer(algo, P):
    roots = [0] if algo in ("bine_lat", "bine_lat_reversed") else sorted({x for x in (0, 1, P - 1, P // 2) if x < P})
    for dt, n in (("float", 37), ("int8", 5), ("double", 1)):
        for root in roots:
            bufs = O.inputs(dt, n, P)
            got = plan_sim.run("bcast", algo, bufs, dt, root=root, in_place=True)
            for r in range(P):
                assert got[r].tobytes() == bufs[root].tobytes(), (algo, P, root, r)


@pytest.mark.parametrize("P", [2, 4, 8, 16])
@pytest.mark.parametrize("algo", BC_LAT)
def test_bcast_message_pattern(algo, P):
    root = 0 if algo in ("bine_lat", "bine_lat_reversed") else P - 1
    sends = 0
    for r in range(P):
        prims, _ = pico_amd.plan("bcast", algo, P, r, count=64, root=root, esz=4, in_place=True)
        recv = [p for p in prims if p["type"] == "RECV"]
        sends += sum(p["type"] == "SEND" for p in prims)
        assert len(recv) == (0 if r == root else 1), (r, recv)
        assert all(p["count"] == 64 for p in prims)
        assert all(p["type"] in ("SEND", "RECV") for p in prims)   # in place: no copies
        # a rank sends only after it has received (group order)
        if recv:
            assert all(p["group"] > recv[0]["group"] for p in prims if p["type"] == "SEND")
        assert len({p["group"] for p in prims}) <= P.bit_length() - 1
    assert sends == P - 1   # a tree: every rank reached once


def test_bine_lat_tree_matches_reference_pi():
    """bcast_bine_lat's parent at each step is pi(rank, step) (:247-249): check
    the plan's peers against the schedule math directly"""
    P, steps = 8, 3
    for r in range(1, P):
        prims, _ = pico_amd.plan("bcast", "bine_lat", P, r, count=8, root=0, esz=4, in_place=True)
        recv = [p for p in prims if p["type"] == "RECV"][0]
        sends = [p for p in prims if p["type"] == "SEND"]
        assert all(p["peer"] != recv["peer"] for p in sends)
    # the root sends at every step
    prims, _ = pico_amd.plan("bcast", "bine_lat", P, 0, count=8, root=0, esz=4, in_place=True)
    assert [p["type"] for p in prims] == ["SEND"] * steps


@pytest.mark.parametrize("algo", BC_LAT)
def test_bcast_errors(algo):
    for P in (3, 5, 6, 12):
        with pytest.raises(pico_amd.BineError) as e:
            pico_amd.plan("bcast", algo, P, 0, count=8, root=0, esz=4, in_place=True)
        assert e.value.status == 2   # ERR_SIZE (MPI_ERR_SIZE)
    if algo in ("bine_lat", "bine_lat_reversed"):
        with pytest.raises(pico_amd.BineError) as e:
            pico_amd.plan("bcast", algo, 4, 1, count=8, root=1, esz=4, in_place=True)
        assert e.value.status == 8   # ERR_ROOT (MPI_ERR_ROOT)


@pytest.mark.parametrize("algo", BC_LAT)
def test_bcast_error_order_and_zero_count(algo):
    """the reference checks the size first, then the root
    (libbine_bcast.c:198-210), before it looks at the count: P = 3 with an
    out-of-range root is MPI_ERR_SIZE, a power-of-two P with root >= P is
    MPI_ERR_ROOT (bine_lat / _reversed: any root != 0; the _new variants hang
    in the reference there -- no rank is the root -- and report MPI_ERR_ROOT
    here), and count = 0 reports the same errors"""
    for count in (0, 8):
        with pytest.raises(pico_amd.BineError) as e:
            pico_amd.plan("bcast", algo, 3, 0, count=count, root=5, esz=4, in_place=True)
        assert e.value.status == 2, (algo, count)
        with pytest.raises(pico_amd.BineError) as e:
            pico_amd.plan("bcast", algo, 4, 0, count=count, root=4, esz=4, in_place=True)
        assert e.value.status == 8, (algo, count)
        with pytest.raises(pico_amd.BineError) as e:
            pico_amd.plan("bcast", algo, 6, 1, count=count, root=0, esz=4, in_place=True)
        assert e.value.status == 2, (algo, count)
    # count = 0 with valid arguments: success, nothing moves
    prims, _ = pico_amd.plan("bcast", algo, 4, 1, count=0, root=0, esz=4, in_place=True)
    assert prims == []


def test_bcast_schedule_race_free():
    from test_schedule import check_race_free
    for algo in BC:
        for P in (2, 4, 8):
            for r in range(P):
                ops, c_join, final_wait = pico_amd.schedule("bcast", algo, P, r, count=999, root=0, esz=4,
                                                            in_place=True, chunk_bytes=256)
                check_race_free(ops, c_join, final_wait, True)


# ---- the bandwidth bcasts (libbine_bcast.c:42, :462, :649; round 5 widening) ----

@pytest.mark.parametrize("P", list(range(1, 17)))
@pytest.mark.parametrize("algo", list(O.BC_BDW))
def test_bcast_bdw_plans_equal_the_replay(algo, P):
    """the planner's per-rank plans, run by the rendezvous simulator, leave
    every rank's buffer exactly as the message-level replay of the reference
    does (oracle.bcast_bdw, itself pinned by the reference's vectors in
    tests/test_oracle.py), return its status where it fails (MPI_ERR_COUNT for
    count < P, MPI_ERR_SIZE / MPI_ERR_ROOT for bine_bdw_static), and where the
    reference crashes (scatter_allgather's wrapped size_t counts) deliver the
    root's buffer; bine_bdw_remap off its domain (root != 0, non-power-of-two
    P, where the reference asserts) is BINE_ERR_ARG"""
    status = {2: 9, 51: 2, 7: 8}   # MPICH code -> bine_status_t
    for n in sorted({1, 3, P, P + 1, 2 * P + 1, 3 * P - 1, 13, 64, 333}):
        for root in sorted({0, 1 % P, P - 1}):
            for dt in ("float", "int8"):
                ins = O.inputs(dt, n, P)
                want, rets = O.bcast_bdw(algo, ins, dt, root)
                try:
                    got, st = plan_sim.run("bcast", algo, ins, dt, root=root, in_place=True), 0
                except pico_amd.BineError as e:
                    got, st = None, e.status
                tag = (algo, P, n, root, dt, rets[:1], st)
                if rets[0] == "crash":
                    if algo == "bine_bdw_remap":
                        assert st == 1, tag
                    else:
                        assert got is not None and all(g.tobytes() == ins[root].tobytes() for g in got), tag
                elif any(rets):
                    assert got is None and status[rets[0]] == st, tag
                else:
                    assert got is not None and all(g.tobytes() == w.tobytes() for g, w in zip(got, want)), tag


def test_bcast_bdw_moves_less_than_the_trees():
    """the point of the bandwidth forms: at P = 8 the root sends 1.75 x the
    buffer (scatter 7/8, allgather 7/8) where a latency tree's root sends it
    log2(P) = 3 times, and the Bine forms receive exactly the buffer once per
    non-root rank; scatter_allgather's recursive doubling re-sends blocks a
    rank already holds (up to 1.375 x)"""
    P, n = 8, 8 * 1024
    for algo in O.BC_BDW:
        sent, recv = [], []
        for r in range(P):
            prims, _ = pico_amd.plan("bcast", algo, P, r, count=n, root=0, esz=4, in_place=True)
            sent.append(sum(p["count"] for p in prims if p["type"] == "SEND"))
            recv.append(sum(p["count"] for p in prims if p["type"] == "RECV"))
        assert sent[0] == 1.75 * n, (algo, sent)
        if algo == "scatter_allgather":
            assert max(recv) <= 1.375 * n, recv
        else:
            assert recv[0] == 0 and all(x == n for x in recv[1:]), (algo, recv)
    tree = pico_amd.plan("bcast", "bine_lat", P, 0, count=n, root=0, esz=4, in_place=True)[0]
    assert sum(p["count"] for p in tree if p["type"] == "SEND") == 3 * n
