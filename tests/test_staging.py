"""Host staging pipelined into the collective (bine_allreduce_staged /
bine_reduce_scatter_staged, libbine.so's path for pico_core's host buffers,
pico_core_allreduce_utils.c:13-25).  CPU: the planner's staging ranges
(pico_amd.stage_plan) run through the plan simulator with the device input
poisoned and the host output assembled only from the device->host pieces,
compared bit for bit with the oracle; plus the structure the executor relies
on (every input piece staged once, before its first toucher; every output
piece copied once, after its last writer) and that the two PCIe directions
overlap (the first copy back is issued long before the last copy in)."""
import numpy as np
import pytest

import pico_amd
import plan_sim
from oracle import oracle as O

SB, RB = 0, 1

# the staged API turns the flat forms on (flat_rs + the chunked allgather);
# algorithms / P without a flat form keep their literal schedules, staged the same way
STAGED = dict(flat_rs=True, flat_ag=2)

AR = ["bine_bdw_remap", "bine_bdw_static", "bine_bdw_remap_segmented", "bine_lat", "rabenseifner",
      "recursivedoubling", "ring", "bine_block_by_block_any_even"]
RS = ["bine_permute_remap", "bine_send_remap", "bine_static", "bine_block_by_block", "recursivehalving",
      "ring", "butterfly", "recursive_distance_doubling", "bine_block_by_block_any_even"]


def _ar_case(algo, P, dtype, n, op, chunk, in_place):
    sb = O.inputs(dtype, n, P)
    want, rets = O.allreduce(algo, sb, dtype, op=op, segsize=256)
    if any(rets):
        return True  # the reference's error: nothing to stage
    got = plan_sim.run("allreduce", algo, sb, dtype, op=op, segsize=256, chunk_bytes=chunk, in_place=in_place,
                       stage=True, **STAGED)
    return all(np.array_equal(got[r], want[r], equal_nan=False) for r in range(P))


def _rs_case(algo, P, dtype, n, op, chunk, in_place):
    even = algo in ("bine_permute_remap",)
    rc = [n // P + 1] * P if even else [n // P + (i % 3) for i in range(P)]
    sb = O.inputs(dtype, sum(rc), P)
    want, rets = O.reduce_scatter(algo, sb, rc, dtype, op=op)
    if any(rets):
        return True
    got = plan_sim.run("reduce_scatter", algo, sb, dtype, op=op, rcounts=rc, chunk_bytes=chunk, in_place=in_place,
                       stage=True, **STAGED)
    return all(np.array_equal(got[r], want[r]) for r in range(P))


@pytest.mark.parametrize("algo", AR)
@pytest.mark.parametrize("P", [2, 3, 4, 8])
def test_staged_allreduce_matches_oracle(algo, P):
    for dtype, n, op in (("float", 997, "sum"), ("int64", 64 * P + 5, "sum"), ("double", 301, "max")):
        for chunk in (64, 512):
            for in_place in (False, True):
                assert _ar_case(algo, P, dtype, n, op, chunk, in_place), (dtype, n, op, chunk, in_place)


@pytest.mark.parametrize("algo", RS)
@pytest.mark.parametrize("P", [2, 4, 8])
def test_staged_reduce_scatter_matches_oracle(algo, P):
    for dtype, n, op in (("float", 997, "sum"), ("int32", 515, "prod")):
        for chunk in (64, 512):
            for in_place in (False, True):
                assert _rs_case(algo, P, dtype, n, op, chunk, in_place), (dtype, n, op, chunk, in_place)


def _touched(prims, buf, in_place):
    """element ranges of `buf` an op reads and writes (SBUF = RBUF in place)"""
    rd, wr = [], []

    def b(x):
        return RB if in_place and x == SB else x

    for p in prims:
        t, n = p["type"], p["count"]
        if t == "SEND":
            rd.append((b(p["src_buf"]), p["src_off"], n))
        elif t == "RECV":
            wr.append((b(p["dst_buf"]), p["dst_off"], n))
        elif t == "REDUCE":
            rd += [(b(p["src_buf"]), p["src_off"], n), (b(p["dst_buf"]), p["dst_off"], n)]
            wr.append((b(p["dst_buf"]), p["dst_off"], n))
        elif t == "REDUCE3":
            rd += [(b(p["src_buf"]), p["src_off"], n), (b(p["aux_buf"]), p["aux_off"], n)]
            wr.append((b(p["dst_buf"]), p["dst_off"], n))
        elif t == "REDUCE_TREE":
            rd += [(b(p["aux_buf"]), p["aux_off"], n), (b(p["src_buf"]), p["src_off"], (p["peer"] - 1) * n)]
            wr.append((b(p["dst_buf"]), p["dst_off"], n))
        else:
            rd.append((b(p["src_buf"]), p["src_off"], n))
            wr.append((b(p["dst_buf"]), p["dst_off"], n))
    keep = lambda L: [(o, o + n) for x, o, n in L if x == buf and n]
    return keep(rd), keep(wr)


def _cover(ranges, size):
    m = np.zeros(size, np.int32)
    for lo, hi in ranges:
        m[lo:hi] += 1
    return m


@pytest.mark.parametrize("coll,algo,P", [("allreduce", "bine_bdw_remap", 8), ("allreduce", "bine_bdw_static", 4),
                                         ("allreduce", "ring", 4), ("allreduce", "ring", 6),
                                         ("allreduce", "bine_bdw_remap_segmented", 6),
                                         ("reduce_scatter", "bine_permute_remap", 8),
                                         ("reduce_scatter", "bine_send_remap", 4)])
def test_stage_ranges_structure(coll, algo, P):
    """every input piece staged exactly once, before (and awaited by) every op
    that touches it; every output piece copied back exactly once, after its
    last writer"""
    n = 4099
    for rank in range(P):
        for in_place in (False, True):
            kw = dict(count=n, esz=4, segsize=1024)
            if coll == "reduce_scatter":
                kw = dict(rcounts=[n // P + (algo != "bine_permute_remap") * (i % 2) for i in range(P)], esz=4)
            ops, _, _ = pico_amd.schedule(coll, algo, P, rank, chunk_bytes=1024, in_place=in_place, **kw, **STAGED)
            h2d, d2h, wait = pico_amd.stage_plan(coll, algo, P, rank, chunk_bytes=1024, in_place=in_place, **kw,
                                                 **STAGED)
            in_buf = RB if in_place else SB
            size = (n if coll == "allreduce" else sum(kw["rcounts"])) + 1
            tin = [_touched(o["prims"], in_buf, in_place) for o in ops]
            tout = [_touched(o["prims"], RB, in_place)[1] for o in ops]
            all_in = _cover([r for rd, wr in tin for r in rd + wr], size)
            staged = _cover([r for v in h2d.values() for r in v], size)
            assert (staged <= 1).all() and ((all_in > 0) == (staged > 0)).all()
            for i, (rd, wr) in enumerate(tin):
                if not rd + wr:
                    continue
                assert wait[i] >= 0
                have = _cover([r for j, v in h2d.items() if j <= wait[i] for r in v], size)
                need = _cover(rd + wr, size)
                assert ((need > 0) <= (have > 0)).all(), (rank, i)
            written = _cover([r for w in tout for r in w], size)
            back = _cover([r for v in d2h.values() for r in v], size)
            assert (back <= 1).all() and ((written > 0) == (back > 0)).all()
            for i, v in d2h.items():  # no later op writes a piece copied back after op i
                later = _cover([r for w in tout[i + 1:] for r in w], size)
                assert all((later[lo:hi] == 0).all() for lo, hi in v)


def test_staged_flat_allreduce_overlaps_both_directions():
    """the chunked flat form (P = 8, 16 chunks of every block): the first copy
    back is issued right after the first chunk's allgather, long before the
    last piece of the input goes in -- so host->device and device->host run
    concurrently; and the allgather leaves chunk by chunk"""
    P, n = 8, 1 << 16
    chunk = n * 4 // P // 16
    for rank in (0, 5):
        h2d, d2h, _ = pico_amd.stage_plan("allreduce", "bine_bdw_remap", P, rank, count=n, esz=4,
                                          chunk_bytes=chunk, **STAGED)
        assert len(d2h) >= 16 and len(h2d) >= 16
        assert min(d2h) < max(h2d) / 4


def test_staging_simulator_negative_controls(monkeypatch):
    """the simulator does see a missing piece: dropping one host->device or one
    device->host piece from the staging ranges breaks the result"""
    P = 8
    sb = O.inputs("float", 997, P)
    want, _ = O.allreduce("bine_bdw_remap", sb, "float")
    orig = pico_amd.stage_plan

    def run():
        got = plan_sim.run("allreduce", "bine_bdw_remap", sb, "float", chunk_bytes=64, stage=True, **STAGED)
        return all(np.array_equal(got[r], want[r]) for r in range(P))

    assert run()
    for kind in (0, 1):
        def cut(*a, kind=kind, **k):
            res = list(orig(*a, **k))
            d = res[kind]
            op = min(d) if kind == 0 else max(d)
            d[op] = d[op][1:]
            return tuple(res)
        monkeypatch.setattr(pico_amd, "stage_plan", cut)
        assert not run(), kind
        monkeypatch.setattr(pico_amd, "stage_plan", orig)
