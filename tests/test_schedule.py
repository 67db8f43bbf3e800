"""The executor's two-stream issue schedule (make_schedule, schedule.cpp),
checked on the host through bine_plan_schedule:

* race freedom -- every pair of ops on different streams (comm stream C:
  exchanges; caller's stream K: reductions / copies) whose memory regions
  conflict (read-after-write, write-after-read, write-after-write) is ordered
  by the happens-before relation the schedule's stream order and event waits
  create (vector clocks);
* the comm stream joins the caller's prior work and the caller's stream ends
  after the last exchange;
* chunking -- the chunked schedule, run in issue order by the rendezvous
  simulator, gives the oracle's (= the reference's) result bit-for-bit.

Race freedom plus issue-order equivalence means every interleaving the GPU may
pick computes the reference's result."""
import numpy as np
import pytest

import pico_amd
import plan_sim
from oracle import oracle as O

SB, RB = 0, 1

AR = ["bine_bdw_remap", "bine_bdw_static", "bine_bdw_remap_segmented", "bine_lat", "ring", "rabenseifner",
      "recursivedoubling", "bine_block_by_block_any_even"]
RS = ["bine_permute_remap", "bine_send_remap", "bine_static", "bine_block_by_block", "bine_block_by_block_any_even",
      "ring", "butterfly", "recursivehalving", "recursive_distance_doubling"]
RD = ["bine_bdw", "bine_lat"]
AG = list(pico_amd.ALGOS["allgather"])


def _regions(p, in_place):
    def reg(b, off, n):
        return ((RB if (in_place and b == SB) else b), off, off + n)
    t, n = p["type"], p["count"]
    if t == "SEND":
        return [reg(p["src_buf"], p["src_off"], n)], []
    if t == "RECV":
        return [], [reg(p["dst_buf"], p["dst_off"], n)]
    if t == "REDUCE":
        d = reg(p["dst_buf"], p["dst_off"], n)
        return [reg(p["src_buf"], p["src_off"], n), d], [d]
    if t == "REDUCE3":
        return [reg(p["src_buf"], p["src_off"], n), reg(p["aux_buf"], p["aux_off"], n)], \
            [reg(p["dst_buf"], p["dst_off"], n)]
    if t == "REDUCE_TREE":  # own leaf at aux, the nl-1 others back to back at src
        return [reg(p["aux_buf"], p["aux_off"], n), reg(p["src_buf"], p["src_off"], (p["peer"] - 1) * n)], \
            [reg(p["dst_buf"], p["dst_off"], n)]
    return [reg(p["src_buf"], p["src_off"], n)], [reg(p["dst_buf"], p["dst_off"], n)]


def _overlap(a, b):
    return any(x[0] == y[0] and x[1] < y[2] and y[1] < x[2] for x in a for y in b)


def check_race_free(ops, c_join, final_wait, in_place):
    n = len(ops)
    # vc[i][s] = newest op of stream s that happens-before-or-is op i
    vc = []
    last = [None, None]
    for i, o in enumerate(ops):
        s = 1 if o["xchg"] else 0
        w = o["wait"]
        assert w < i
        if w >= 0:
            assert ops[w]["xchg"] != o["xchg"], "wait on own stream"
        v = [-1, -1]
        for src in (last[s], w if w >= 0 else None):
            if src is not None:
                v = [max(v[0], vc[src][0]), max(v[1], vc[src][1])]
        v[s] = i
        vc.append(v)
        last[s] = i
    regs = []
    for o in ops:
        rd, wr = [], []
        for p in o["prims"]:
            a, b = _regions(p, in_place)
            rd += a
            wr += b
        regs.append((rd, wr))
    for j in range(n):
        sj = 1 if ops[j]["xchg"] else 0
        for i in range(j):
            si = 1 if ops[i]["xchg"] else 0
            if si == sj:
                continue
            (ri, wi), (rj, wj) = regs[i], regs[j]
            if _overlap(wi, rj) or _overlap(wi, wj) or _overlap(ri, wj):
                assert vc[j][si] >= i, f"race: op {i} ({ops[i]['prims'][0]['type']}) vs op {j}"
    xs = [i for i, o in enumerate(ops) if o["xchg"]]
    if xs:
        assert c_join
        ks = [i for i, o in enumerate(ops) if not o["xchg"]]
        covered = max(final_wait, vc[ks[-1]][1] if ks else -1)
        assert covered >= xs[-1], "caller's stream does not wait for the last exchange"


def _cases():
    for P in (2, 3, 4, 5, 6, 8, 16):
        for a in AR:
            yield "allreduce", a, P
        for a in RS:
            yield "reduce_scatter", a, P
        for a in RD:
            yield "reduce", a, P
        for a in AG:
            yield "allgather", a, P


@pytest.mark.parametrize("chunk", [0, 64, 4096])
@pytest.mark.parametrize("in_place", [False, True])
def test_schedules_race_free(chunk, in_place):
    checked = 0
    for coll, algo, P in _cases():
        for rank in range(P):
            kw = dict(count=1003, esz=4, segsize=128, in_place=in_place)
            if coll == "reduce_scatter":
                kw = dict(rcounts=[37 + (i % 3) * (algo != "bine_permute_remap") for i in range(P)], esz=4,
                          in_place=in_place)
            if coll == "allgather":
                kw = dict(count=101, esz=4, in_place=in_place)
            try:
                ops, cj, fw = pico_amd.schedule(coll, algo, P, rank, chunk_bytes=chunk, **kw)
            except pico_amd.BineError:
                continue
            check_race_free(ops, cj, fw, in_place)
            checked += 1
    assert checked > 300


def test_chunking_overlaps_steps():
    """With chunks, the first chunk of a step waits for the reduction of the
    region it sends, not for the whole previous step."""
    ops, _, _ = pico_amd.schedule("allreduce", "bine_bdw_remap", 8, 3, count=1 << 16, chunk_bytes=4096)
    red = [i for i, o in enumerate(ops) if not o["xchg"]]
    xch = [i for i, o in enumerate(ops) if o["xchg"]]
    # some exchange is issued while a reduction issued earlier is not waited for
    assert any(0 <= ops[j]["wait"] < max(i for i in red if i < j) for j in xch if any(i < j for i in red))


@pytest.mark.parametrize("coll,algo,P", [
    ("allreduce", "bine_bdw_remap", 4), ("allreduce", "bine_bdw_static", 8), ("allreduce", "rabenseifner", 6),
    ("allreduce", "bine_bdw_remap_segmented", 4), ("allreduce", "ring", 5),
    ("reduce_scatter", "bine_permute_remap", 8), ("reduce_scatter", "bine_static", 4),
    ("reduce_scatter", "ring", 3), ("reduce_scatter", "recursivehalving", 8),
    ("reduce", "bine_bdw", 8),
    ("allgather", "bine_permute_remap", 8), ("allgather", "bine_send_static", 8), ("allgather", "ring", 5),
    ("allgather", "k_bruck", 6), ("allgather", "bine_2_blocks", 8), ("allgather", "recursivedoubling", 4),
    ("allgather", "sparbit", 6),
])
@pytest.mark.parametrize("chunk", [16, 200])
def test_chunked_schedule_matches_oracle(coll, algo, P, chunk):
    dtype = "float"
    if coll == "allgather":
        assert _run_relay(coll, algo, P, chunk, 0)
        return
    if coll == "reduce_scatter":
        rc = [29 + 3 * (i % 2) * (algo != "bine_permute_remap") for i in range(P)]  # permute: equal blocks
        sb = O.inputs(dtype, sum(rc), P)
        want = O.reduce_scatter(algo, sb, rc, dtype)[0]
        got = plan_sim.run(coll, algo, sb, dtype, rcounts=rc, chunk_bytes=chunk)
        for r in range(P):
            assert np.array_equal(got[r], want[r])
        return
    sb = O.inputs(dtype, 997, P)
    if coll == "allreduce":
        want = O.allreduce(algo, sb, dtype, segsize=64)[0]
        got = plan_sim.run(coll, algo, sb, dtype, segsize=64, chunk_bytes=chunk)
        for r in range(P):
            assert np.array_equal(got[r], want[r])
    else:
        want = O.reduce(algo, sb, dtype)[0]
        got = plan_sim.run(coll, algo, sb, dtype, chunk_bytes=chunk)
        assert np.array_equal(got[0], want)


# ---- multi-link relay ---------------------------------------------------------

RELAY_CASES = [
    ("allreduce", "bine_bdw_remap", 4), ("allreduce", "bine_bdw_remap", 8), ("allreduce", "bine_bdw_static", 8),
    ("allreduce", "rabenseifner", 6), ("allreduce", "bine_lat", 8), ("allreduce", "ring", 5), ("allreduce", "rabenseifner", 8),
    ("allreduce", "bine_bdw_remap_segmented", 8), ("allreduce", "recursivedoubling", 4),
    ("reduce_scatter", "bine_permute_remap", 8), ("reduce_scatter", "bine_send_remap", 4),
    ("reduce_scatter", "bine_static", 8), ("reduce_scatter", "recursivehalving", 8), ("reduce_scatter", "ring", 6),
    ("reduce_scatter", "butterfly", 8),
    ("reduce", "bine_bdw", 8),
    ("allgather", "bine_permute_remap", 8), ("allgather", "bine_send_static", 8), ("allgather", "ring", 5),
    ("allgather", "k_bruck", 6), ("allgather", "bine_2_blocks", 8), ("allgather", "recursivedoubling", 4),
    ("allgather", "sparbit", 6),
]


def _run_relay(coll, algo, P, chunk, relay, n=997):
    dtype = "float"
    if coll == "allgather":
        sb = O.inputs(dtype, n // P + 1, P)
        want = O.allgather(algo, sb, dtype)[0]
        got = plan_sim.run(coll, algo, sb, dtype, chunk_bytes=chunk, relay=relay)
        return all(np.array_equal(got[r], want[r]) for r in range(P))
    if coll == "reduce_scatter":
        rc = [n // P + (i % 2) * (algo != "bine_permute_remap") for i in range(P)]
        sb = O.inputs(dtype, sum(rc), P)
        want = O.reduce_scatter(algo, sb, rc, dtype)[0]
        got = plan_sim.run(coll, algo, sb, dtype, rcounts=rc, chunk_bytes=chunk, relay=relay)
        return all(np.array_equal(got[r], want[r]) for r in range(P))
    sb = O.inputs(dtype, n, P)
    if coll == "allreduce":
        want = O.allreduce(algo, sb, dtype, segsize=256)[0]
        got = plan_sim.run(coll, algo, sb, dtype, segsize=256, chunk_bytes=chunk, relay=relay)
        return all(np.array_equal(got[r], want[r]) for r in range(P))
    want = O.reduce(algo, sb, dtype)[0]
    got = plan_sim.run(coll, algo, sb, dtype, chunk_bytes=chunk, relay=relay)
    return np.array_equal(got[0], want)


@pytest.mark.parametrize("coll,algo,P", RELAY_CASES)
@pytest.mark.parametrize("chunk,relay", [(0, 4), (256, 4), (1024, 16)])
def test_relay_schedule_matches_oracle(coll, algo, P, chunk, relay):
    assert _run_relay(coll, algo, P, chunk, relay)


@pytest.mark.parametrize("coll,algo,P", RELAY_CASES)
def test_relay_schedules_race_free(coll, algo, P):
    for rank in range(P):
        kw = dict(count=4099, esz=4, segsize=512)
        if coll == "reduce_scatter":
            kw = dict(rcounts=[500 + (i % 3) * (algo != "bine_permute_remap") for i in range(P)], esz=4)
        if coll == "allgather":
            kw = dict(count=513, esz=4)
        for chunk in (0, 1024):
            ops, cj, fw = pico_amd.schedule(coll, algo, P, rank, chunk_bytes=chunk, relay_min_bytes=8, **kw)
            check_race_free(ops, cj, fw, False)


def _link_loads(coll, algo, P, **kw):
    """bytes per directed link (src, dst) summed over each rank's schedule"""
    loads = {}
    for r in range(P):
        ops, _, _ = pico_amd.schedule(coll, algo, P, r, **kw)
        for o in ops:
            for p in o["prims"]:
                if p["type"] == "SEND":
                    loads[(r, p["peer"])] = loads.get((r, p["peer"]), 0) + p["count"]
    return loads


def test_relay_spreads_steps_over_all_links():
    """remap allreduce at P=8: direct execution puts each step on one link per
    rank (3 peers per rank over the whole collective); relay uses all 7 links
    and the busiest link carries ~4x less than direct execution's busiest."""
    n = 1 << 20
    kw = dict(count=n, esz=4, chunk_bytes=1 << 16)
    direct = _link_loads("allreduce", "bine_bdw_remap", 8, **kw)
    relay = _link_loads("allreduce", "bine_bdw_remap", 8, relay_min_bytes=1024, **kw)
    assert {len({d for (s, d) in direct if s == r}) for r in range(8)} == {3}
    assert {len({d for (s, d) in relay if s == r}) for r in range(8)} == {7}
    assert sum(relay.values()) > sum(direct.values())  # two-hop parts cost extra bytes
    # direct execution uses one link at a time: its time ~ a rank's total bytes;
    # relay keeps all links busy: time ~ the busiest link's bytes (P/2 = 4x less)
    direct_time = max(sum(v for (s, d), v in direct.items() if s == r) for r in range(8))
    assert max(relay.values()) * 3.9 < direct_time


def test_relay_off_for_non_permutation_steps():
    """block-by-block exchanges of several blocks per group are left as they
    are; only its final one-block step is relayed"""
    a, _, _ = pico_amd.schedule("reduce_scatter", "bine_block_by_block", 8, 0, rcounts=[64] * 8)
    b, _, _ = pico_amd.schedule("reduce_scatter", "bine_block_by_block", 8, 0, rcounts=[64] * 8,
                                relay_min_bytes=4)
    multi = [i for i, o in enumerate(a) if o["xchg"] and len(o["prims"]) > 2]
    assert multi and a[:max(multi) + 1] == b[:max(multi) + 1]
    assert len(b) > len(a)


# ---- flat allgather phase ------------------------------------------------------

FLAT_AG = ["bine_bdw_remap", "bine_bdw_static", "bine_bdw_remap_segmented", "rabenseifner"]


@pytest.mark.parametrize("algo", FLAT_AG)
@pytest.mark.parametrize("P", [2, 4, 8, 16])
@pytest.mark.parametrize("chunk,relay", [(0, 0), (256, 0), (256, 4)])
def test_flat_allgather_matches_oracle(algo, P, chunk, relay):
    """one all-peers exchange replaces the mirrored allgather: bit-identical to
    the reference (the reduce-scatter and its reduction order are untouched)"""
    for dtype, n in (("float", 997), ("int64", 64 * P + 5), ("double", 3)):
        sb = O.inputs(dtype, n, P)
        want, rets = O.allreduce(algo, sb, dtype, segsize=256)
        for in_place in (False, True):
            got = plan_sim.run("allreduce", algo, sb, dtype, segsize=256, chunk_bytes=chunk, relay=relay,
                               flat_ag=True, in_place=in_place)
            for r in range(P):
                assert np.array_equal(got[r], want[r]), (algo, P, dtype, in_place, r)


@pytest.mark.parametrize("algo", FLAT_AG)
@pytest.mark.parametrize("P", [4, 8])
def test_flat_allgather_schedule_race_free_and_one_step(algo, P):
    for rank in range(P):
        for in_place in (False, True):
            ops, cj, fw = pico_amd.schedule("allreduce", algo, P, rank, count=4099, esz=4, chunk_bytes=1024,
                                            segsize=256, in_place=in_place, flat_ag=True)
            check_race_free(ops, cj, fw, in_place)
            # the allgather phase is the last exchange: one group, all P-1 peers
            last = [o for o in ops if o["xchg"]][-1]
            assert {p["peer"] for p in last["prims"] if p["type"] == "SEND"} == set(range(P)) - {rank}
            assert {p["peer"] for p in last["prims"] if p["type"] == "RECV"} == set(range(P)) - {rank}


def test_flat_allgather_not_applied_where_it_does_not_fit():
    """non-power-of-two segmented (folded ranks) and multi-tree instances keep
    their own allgather; other algorithms ignore the flag"""
    P = 6
    sb = O.inputs("float", 1001, P)
    want, _ = O.allreduce("bine_bdw_remap_segmented", sb, "float", segsize=256)
    got = plan_sim.run("allreduce", "bine_bdw_remap_segmented", sb, "float", segsize=256, chunk_bytes=0, flat_ag=True)
    assert all(np.array_equal(g, w) for g, w in zip(got, want))
    sb = O.inputs("float", 1001, P)
    want, _ = O.allreduce("rabenseifner", sb, "float")
    got = plan_sim.run("allreduce", "rabenseifner", sb, "float", chunk_bytes=0, flat_ag=True)
    assert all(np.array_equal(g, w) for g, w in zip(got, want))
    for algo in ("ring", "bine_lat", "recursivedoubling"):
        a = pico_amd.schedule("allreduce", algo, 8, 3, count=4099, esz=4, chunk_bytes=1024)
        b = pico_amd.schedule("allreduce", algo, 8, 3, count=4099, esz=4, chunk_bytes=1024, flat_ag=True)
        assert a == b


def _link_time(coll, algo, P, **kw):
    """link-time model of a schedule: exchange ops run one after another on the
    comm stream, the links of one op in parallel -> sum over ops of the busiest
    directed link's bytes (max over ranks, op by op)"""
    per_rank = []
    for r in range(P):
        ops, _, _ = pico_amd.schedule(coll, algo, P, r, **kw)
        t = []
        for o in ops:
            if not o["xchg"]:
                continue
            link = {}
            for p in o["prims"]:
                if p["type"] in ("SEND", "RECV"):
                    k = (p["type"], p["peer"])
                    link[k] = link.get(k, 0) + p["count"]
            t.append(max(link.values()))
        per_rank.append(t)
    return sum(max(ts) for ts in zip(*per_rank))


def test_flat_allgather_link_time_model():
    """P = 8, remap: in units of S/link the literal schedule takes 1.75 (RS 0.875
    + AG 0.875); the flat allgather costs 0.125 instead of 0.875 -> 1.0; with
    the relayed reduce-scatter (0.21875) 0.34375 instead of relay's 0.4375"""
    n = 1 << 20
    kw = dict(count=n, esz=4, chunk_bytes=1 << 16)
    direct = _link_time("allreduce", "bine_bdw_remap", 8, **kw)
    flat = _link_time("allreduce", "bine_bdw_remap", 8, flat_ag=True, **kw)
    relay = _link_time("allreduce", "bine_bdw_remap", 8, relay_min_bytes=1024, **kw)
    relay_flat = _link_time("allreduce", "bine_bdw_remap", 8, relay_min_bytes=1024, flat_ag=True, **kw)
    assert abs(direct / n - 1.75) < 0.01
    assert abs(flat / n - 1.0) < 0.01
    assert abs(relay / n - 0.4375) < 0.02
    assert abs(relay_flat / n - 0.34375) < 0.02


@pytest.mark.parametrize("P", [2, 4, 8, 16])
def test_flat_gather_reduce_bdw_matches_oracle(P):
    """reduce_bine_bdw with the gather tree replaced by one step into the root:
    the reference's bits at the root"""
    for dtype, n in (("float", 997), ("int64", 64 * P + 5), ("double", 3)):
        sb = O.inputs(dtype, n, P)
        want, _ = O.reduce("bine_bdw", sb, dtype)
        for in_place in (False, True):
            got = plan_sim.run("reduce", "bine_bdw", sb, dtype, chunk_bytes=256, relay=4, flat_ag=True,
                               in_place=in_place)
            assert np.array_equal(got[0], want), (P, dtype, in_place)
        for rank in range(P):
            ops, cj, fw = pico_amd.schedule("reduce", "bine_bdw", P, rank, count=n, esz=8, chunk_bytes=256,
                                            flat_ag=True)
            check_race_free(ops, cj, fw, False)


# ---- flat reduce-scatter phase ----------------------------------------------------

FLAT_RS = [("allreduce", "bine_bdw_remap"), ("allreduce", "bine_bdw_static"),
           ("allreduce", "bine_bdw_remap_segmented"), ("reduce_scatter", "bine_permute_remap"),
           ("reduce_scatter", "bine_send_remap"), ("reduce_scatter", "bine_static"),
           ("reduce_scatter", "bine_block_by_block"), ("reduce", "bine_bdw"),
           ("allreduce", "rabenseifner"), ("reduce_scatter", "recursivehalving"), ("reduce", "bine_lat"),
           ("allreduce", "bine_lat"), ("allreduce", "recursivedoubling"),
           ("reduce_scatter", "recursive_distance_doubling"), ("reduce_scatter", "butterfly"),
           ("allreduce", "bine_block_by_block_any_even"), ("reduce_scatter", "bine_block_by_block_any_even"),
           ("allreduce", "ring"), ("reduce_scatter", "ring")]


def _flat_rs_case(coll, algo, P, dtype, n, op, chunk, in_place, flat_ag):
    if coll == "allreduce":
        sb = O.inputs(dtype, n, P)
        want, _ = O.allreduce(algo, sb, dtype, op=op, segsize=256)
        got = plan_sim.run(coll, algo, sb, dtype, op=op, segsize=256, chunk_bytes=chunk, flat_rs=True,
                           flat_ag=flat_ag, in_place=in_place)
        return all(np.array_equal(got[r], want[r]) for r in range(P))
    if coll == "reduce_scatter":
        rc = [n // P + 1] * P if algo == "bine_permute_remap" else [n // P + (i % 3) for i in range(P)]
        sb = O.inputs(dtype, sum(rc), P)
        want, _ = O.reduce_scatter(algo, sb, rc, dtype, op=op)
        got = plan_sim.run(coll, algo, sb, dtype, op=op, rcounts=rc, chunk_bytes=chunk, flat_rs=True,
                           in_place=in_place)
        return all(np.array_equal(got[r], want[r]) for r in range(P))
    sb = O.inputs(dtype, n, P)
    want, _ = O.reduce(algo, sb, dtype, op=op)
    got = plan_sim.run(coll, algo, sb, dtype, op=op, chunk_bytes=chunk, flat_rs=True, flat_ag=flat_ag,
                       in_place=in_place)
    return np.array_equal(got[0], want)


@pytest.mark.parametrize("coll,algo", FLAT_RS)
@pytest.mark.parametrize("P", [2, 4, 8, 16])
def test_flat_reduce_scatter_matches_oracle(coll, algo, P):
    """one all-peers exchange + the reference's reduction tree per block
    (REDUCE_TREE) gives the reference's bits: fp and int, SUM / MAX / PROD,
    ragged blocks, chunked, in place, with and without the flat allgather"""
    for dtype, n, op in (("float", 997, "sum"), ("int64", 64 * P + 5, "sum"), ("double", 3, "sum"),
                         ("float", 1001, "max"), ("int32", 515, "prod")):
        for chunk in (0, 64):
            for in_place in (False, True):
                for flat_ag in ((False, True, 2) if coll != "reduce_scatter" else (False,)):
                    assert _flat_rs_case(coll, algo, P, dtype, n, op, chunk, in_place, flat_ag), \
                        (dtype, n, op, chunk, in_place, flat_ag)


@pytest.mark.parametrize("coll,algo", FLAT_RS)
@pytest.mark.parametrize("P", [4, 8])
def test_flat_reduce_scatter_race_free_and_one_hop(coll, algo, P):
    """race-free under chunking; every exchange of the reduce-scatter phase
    talks to all P-1 peers; one REDUCE_TREE of P leaves per chunk"""
    for rank in range(P):
        for in_place in (False, True):
            kw = dict(count=4099, esz=4, segsize=256)
            if coll == "reduce_scatter":
                kw = dict(rcounts=[513 + (i % 2) * (algo != "bine_permute_remap") for i in range(P)], esz=4)
            ops, cj, fw = pico_amd.schedule(coll, algo, P, rank, chunk_bytes=1024, in_place=in_place, flat_rs=True,
                                            **kw)
            check_race_free(ops, cj, fw, in_place)
            trees = [p for o in ops for p in o["prims"] if p["type"] == "REDUCE_TREE"]
            assert all(p["peer"] == P for p in trees)
            if algo != "ring":  # the rings fold their chain with pairwise reductions
                assert trees or ((coll, algo) == ("reduce", "bine_lat") and rank != 0)  # the root's tree
                assert not any(p["type"] in ("REDUCE", "REDUCE3") for o in ops for p in o["prims"])
            first = [o for o in ops if o["xchg"]][0]
            sends = {p["peer"] for p in first["prims"] if p["type"] == "SEND"}
            if (coll, algo) == ("reduce", "bine_lat"):  # every rank straight to the root
                assert sends == ({0} if rank else set())
            else:
                assert sends == set(range(P)) - {rank}


FLAT_AG_CHUNKED = [a for c, a in FLAT_RS if c == "allreduce" and a not in ("bine_lat", "recursivedoubling")]


@pytest.mark.parametrize("algo", FLAT_AG_CHUNKED)
@pytest.mark.parametrize("P", [2, 4, 8])
def test_flat_ag_chunked_race_free_and_interleaved(algo, P):
    """flat_ag = 2: the allgather is cut with the reduce-scatter's chunks.
    Race-free; every allgather exchange moves one chunk of every block (all
    P-1 peers); the k-th allgather exchange follows the (k+1)-th reduce-scatter
    exchange; the allgather moves exactly the bytes of the one-exchange form"""
    n, ch = 4099, 1024
    for rank in range(P):
        for in_place in (False, True):
            kw = dict(count=n, esz=4, segsize=256, chunk_bytes=ch, in_place=in_place, flat_rs=True)
            ops, cj, fw = pico_amd.schedule("allreduce", algo, P, rank, flat_ag=2, **kw)
            check_race_free(ops, cj, fw, in_place)
            one, _, _ = pico_amd.schedule("allreduce", algo, P, rank, flat_ag=True, **kw)
            def ag_sends(o_):  # (peer, elements) of every RBUF -> RBUF send
                return [(p["peer"], p["count"]) for x in o_ if x["xchg"] for p in x["prims"]
                        if p["type"] == "SEND" and p["src_buf"] == RB]
            if in_place:  # the input is RBUF too: compare the totals only
                continue
            per_peer = lambda L: {q: sum(c for p_, c in L if p_ == q) for q, _ in L}
            assert per_peer(ag_sends(ops)) == per_peer(ag_sends(one))
            xs = [o for o in ops if o["xchg"]]
            # reduce-scatter exchanges send SBUF; allgather exchanges only move RBUF
            rs = [i for i, o in enumerate(xs) if any(p["type"] == "SEND" and p["src_buf"] == SB
                                                     for p in o["prims"])]
            ag = [i for i in range(len(xs)) if i not in rs]
            assert len(rs) >= 2 and len(ag) == len(rs)
            for k in range(len(rs) - 1):
                assert rs[k + 1] < ag[k]
            for i in ag:
                assert all(p["src_buf" if p["type"] == "SEND" else "dst_buf"] == RB for p in xs[i]["prims"])
                got = {p["peer"] for p in xs[i]["prims"] if p["type"] == "RECV"}
                assert got and got <= set(range(P)) - {rank}  # (ragged blocks: a short block may be done)
            assert {p["peer"] for p in xs[ag[0]]["prims"] if p["type"] == "RECV"} == set(range(P)) - {rank}


def test_flat_reduce_scatter_not_applied_where_it_does_not_fit():
    """non-power-of-two P and the other algorithms keep their literal schedule"""
    for coll, algo, P in (("allreduce", "bine_bdw_remap_segmented", 6), ("allreduce", "ring", 6),
                          ("allreduce", "rabenseifner", 6), ("reduce_scatter", "recursivehalving", 6),
                          ("reduce_scatter", "ring", 6)):
        kw = dict(rcounts=[100] * P) if coll == "reduce_scatter" else dict(count=4099)
        a = pico_amd.schedule(coll, algo, P, 1, esz=4, chunk_bytes=1024, segsize=256, **kw)
        b = pico_amd.schedule(coll, algo, P, 1, esz=4, chunk_bytes=1024, segsize=256, flat_rs=True, **kw)
        assert a == b


def test_flat_reduce_scatter_link_time_model():
    """P = 8, remap allreduce in units of S / link: flat RS + flat AG = 0.125 +
    0.125 = 0.25 -- the multi-tree mode's link time, but bit-identical to the
    reference; C4's reduce-scatter 0.125 (vs 0.875 literal)"""
    n = 1 << 20
    kw = dict(count=n, esz=4, chunk_bytes=1 << 16)
    assert abs(_link_time("allreduce", "bine_bdw_remap", 8, flat_rs=True, flat_ag=True, **kw) / n - 0.25) < 0.01
    assert abs(_link_time("allreduce", "bine_bdw_remap", 8, flat_rs=True, **kw) / n - 1.0) < 0.01
    rk = dict(rcounts=[n // 8] * 8, esz=4, chunk_bytes=1 << 16)
    assert abs(_link_time("reduce_scatter", "bine_permute_remap", 8, **rk) / n - 0.875) < 0.01
    assert abs(_link_time("reduce_scatter", "bine_permute_remap", 8, flat_rs=True, **rk) / n - 0.125) < 0.01


def test_flat_block_by_block_keeps_the_swapped_last_step():
    """reduce_scatter_bine_block_by_block reduces (own, received) at its last
    step (libbine_reduce_scatter.c:1143), the other steps (received, own): the
    flat tree swaps its top level.  With signed zeros and NaNs MAX / MIN see
    the difference -- the flat schedule matches the reference, and the same
    schedule with the swap bit cleared does not (negative control)"""
    P = 8
    rng = np.random.default_rng(3)
    vals = np.array([0.0, -0.0, np.nan, 1.0, -1.0], np.float32)
    rc = [5 + (i % 2) for i in range(P)]
    sb = [rng.choice(vals, sum(rc)).astype(np.float32) for _ in range(P)]
    orig = plan_sim.scheduled_prims

    def unswapped(*a, **k):
        prims, info = orig(*a, **k)
        for p in prims:
            if p["type"] == "REDUCE_TREE":
                p["flags"] &= 0xFF
        return prims, info
    for op in ("max", "min"):
        want, _ = O.reduce_scatter("bine_block_by_block", sb, rc, "float", op=op)
        got = plan_sim.run("reduce_scatter", "bine_block_by_block", sb, "float", op=op, rcounts=rc, chunk_bytes=0,
                           flat_rs=True)
        assert all(g.tobytes() == w.tobytes() for g, w in zip(got, want)), op
        plan_sim.scheduled_prims = unswapped
        try:
            bad = plan_sim.run("reduce_scatter", "bine_block_by_block", sb, "float", op=op, rcounts=rc,
                               chunk_bytes=0, flat_rs=True)
        finally:
            plan_sim.scheduled_prims = orig
        assert not all(g.tobytes() == w.tobytes() for g, w in zip(bad, want)), op


@pytest.mark.parametrize("P", [2, 3, 4, 6, 8, 16])
def test_flat_allgather_family(P):
    """allgather family with the flat flag: the algorithm's own plan decides
    the status, a successful one becomes one all-peers exchange -- the
    reference's blocks in the reference's places; in place keeps the literal
    algorithm (each has its own in-place input layout)"""
    for algo in AG:
        for dt, n in (("float", 7), ("int8", 33), ("double", 1)):
            sb = O.inputs(dt, n, P)
            try:
                lit = plan_sim.run("allgather", algo, sb, dt, chunk_bytes=64)
            except pico_amd.BineError as e:
                with pytest.raises(pico_amd.BineError) as f:
                    plan_sim.run("allgather", algo, sb, dt, chunk_bytes=64, flat_ag=True)
                assert f.value.status == e.status
                continue
            got = plan_sim.run("allgather", algo, sb, dt, chunk_bytes=64, flat_ag=True)
            want, _ = O.allgather(algo, sb, dt)
            assert all(np.array_equal(g, w) for g, w in zip(got, want)), (algo, dt)
            assert all(np.array_equal(g, w) for g, w in zip(lit, want)), (algo, dt)
            ops, _, _ = pico_amd.schedule("allgather", algo, P, 1, count=n, esz=4, chunk_bytes=64, flat_ag=True)
            assert len([o for o in ops if o["xchg"]]) == 1
