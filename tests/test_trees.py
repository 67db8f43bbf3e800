"""Multi-tree mode (pico_amd/csrc/trees.cpp): P-1 relabelled instances of the
allreduce schedule on P-1 slices, pairing the ranks along edge-disjoint
matchings at every step.

* the relabellings: at every step the instances' pairings are pairwise
  edge-disjoint and together cover every link of the node;
* results: each slice equals, bit for bit, the oracle's restatement of the
  reference run on that slice with the inputs permuted by the relabelling
  (virtual rank v holds physical rank sigma_k[v]'s data); integer results equal
  the reference's own allreduce bit for bit; floating point stays within
  rounding of it;
* the chunked two-stream schedules of tree plans are race-free and deadlock-free.
"""
import numpy as np
import pytest

import pico_amd
import plan_sim
from oracle import oracle as O
from test_schedule import check_race_free

RELABEL = {
    4: [[0, 1, 2, 3], [0, 2, 3, 1], [0, 3, 1, 2]],
    8: [[0, 1, 2, 3, 4, 5, 6, 7], [0, 2, 3, 1, 4, 6, 7, 5], [0, 3, 1, 6, 2, 5, 7, 4], [0, 4, 7, 2, 5, 1, 6, 3],
        [0, 5, 3, 7, 1, 4, 6, 2], [0, 6, 3, 5, 4, 2, 7, 1], [0, 7, 3, 4, 2, 1, 5, 6]],
}
ALGOS = ["bine_bdw_remap", "bine_bdw_static", "bine_lat", "ring", "rabenseifner", "recursivedoubling",
         "bine_bdw_remap_segmented", "bine_block_by_block_any_even"]


@pytest.mark.parametrize("P", [4, 8])
def test_relabellings_cover_every_link_once_per_step(P):
    steps = P.bit_length() - 1
    for s in range(steps):
        edges = set()
        for sig in RELABEL[P]:
            for r in range(P):
                e = frozenset((sig[r], sig[O.pi(r, s, P)]))
                assert len(e) == 2
                edges.add((e, tuple(sig)))
        per_edge = {}
        for e, k in edges:
            per_edge.setdefault(e, set()).add(k)
        assert len(per_edge) == P * (P - 1) // 2              # every link used ...
        assert all(len(v) == 1 for v in per_edge.values())    # ... by exactly one instance


def _slices(n, P):
    T = P - 1
    base = n // T // 64 * 64
    return [(k * base, (n - k * base) if k == T - 1 else base) for k in range(T)]


def relabelled_oracle(algo, sb, dtype, segsize=0):
    """what multi-tree mode must compute: per slice, the reference schedule on
    relabelled ranks"""
    P, n = len(sb), sb[0].size
    out = [np.zeros(n, sb[0].dtype) for _ in range(P)]
    for k, (off, ln) in enumerate(_slices(n, P)):
        sig = RELABEL[P][k]
        virt = [np.ascontiguousarray(sb[sig[v]][off:off + ln]) for v in range(P)]
        res, rets = O.allreduce(algo, virt, dtype, segsize=segsize, ref_bugs=False)
        assert not any(rets)
        for v in range(P):
            out[sig[v]][off:off + ln] = res[v]
    return out


@pytest.mark.parametrize("algo", ALGOS)
@pytest.mark.parametrize("P", [4, 8])
@pytest.mark.parametrize("chunk", [0, 512])
def test_tree_plans_match_relabelled_oracle(algo, P, chunk):
    n = 64 * (P - 1) * 3 + 37
    for dtype in ("float", "int64"):
        sb = O.inputs(dtype, n, P)
        want = relabelled_oracle(algo, sb, dtype, segsize=256)
        got = plan_sim.run("allreduce", algo, sb, dtype, segsize=256, chunk_bytes=chunk, trees=True)
        for r in range(P):
            assert np.array_equal(got[r], want[r]), (algo, P, dtype, r)
        if dtype == "int64":  # integers: identical to the reference itself
            ref, _ = O.allreduce(algo, sb, dtype, segsize=256, ref_bugs=False)
            assert all(np.array_equal(g, w) for g, w in zip(got, ref))
        else:                 # floats: within rounding of the reference
            ref, _ = O.allreduce(algo, sb, dtype, segsize=256, ref_bugs=False)
            assert max(float(np.max(np.abs(g - w))) for g, w in zip(got, ref)) <= P * 1e-4


@pytest.mark.parametrize("P", [4, 8])
def test_tree_plan_uses_every_peer_each_step(P):
    prims, _ = pico_amd.plan("allreduce", "bine_bdw_remap", P, 0, count=1 << 16)
    ops, _, _ = pico_amd.schedule("allreduce", "bine_bdw_remap", P, 0, count=1 << 16, trees=True)
    groups = [o for o in ops if o["xchg"]]
    assert len(groups) == 2 * (P.bit_length() - 1)
    for o in groups:
        assert sorted({p["peer"] for p in o["prims"] if p["type"] == "SEND"}) == [x for x in range(P) if x]


@pytest.mark.parametrize("P", [4, 8])
@pytest.mark.parametrize("chunk", [0, 4096])
def test_tree_schedules_race_free(P, chunk):
    for algo in ALGOS:
        for r in range(P):
            for ip in (False, True):
                ops, cj, fw = pico_amd.schedule("allreduce", algo, P, r, count=64 * (P - 1) * 5 + 3, esz=4,
                                                segsize=512, in_place=ip, chunk_bytes=chunk, trees=True)
                check_race_free(ops, cj, fw, ip)


def test_small_counts_and_other_sizes_fall_back():
    # below one 64-element slice per instance, or P without relabellings: the
    # ordinary plan (bit-exact with the reference)
    a, _, _ = pico_amd.schedule("allreduce", "bine_bdw_remap", 8, 0, count=100, trees=True)
    b, _, _ = pico_amd.schedule("allreduce", "bine_bdw_remap", 8, 0, count=100)
    assert a == b
    a, _, _ = pico_amd.schedule("allreduce", "bine_bdw_remap", 16, 0, count=1 << 16, trees=True)
    b, _, _ = pico_amd.schedule("allreduce", "bine_bdw_remap", 16, 0, count=1 << 16)
    assert a == b


def relabelled_rs_oracle(sb, rc, dtype):
    """multi-tree reduce_scatter_bine_permute_remap: instance k reduces
    sub-range k of every block, virtual block u = physical block sigma_k[u]"""
    P = len(sb)
    T = P - 1
    disp = np.concatenate([[0], np.cumsum(rc)])
    out = [np.zeros(rc[r], sb[0].dtype) for r in range(P)]

    def sl(n, k):
        base = n // T // 64 * 64
        return k * base, (n - k * base) if k == T - 1 else base

    for k in range(T):
        sig = RELABEL[P][k]
        vr = [sl(rc[sig[u]], k)[1] for u in range(P)]
        virt = []
        for v in range(P):
            parts = []
            for u in range(P):
                j = sig[u]
                o, ln = sl(rc[j], k)
                parts.append(sb[sig[v]][disp[j] + o:disp[j] + o + ln])
            virt.append(np.ascontiguousarray(np.concatenate(parts)))
        res, rets = O.reduce_scatter("bine_permute_remap", virt, vr, dtype)
        assert not any(rets)
        for v in range(P):
            r = sig[v]
            o, ln = sl(rc[r], k)
            out[r][o:o + ln] = res[v]
    return out


@pytest.mark.parametrize("P", [4, 8])
@pytest.mark.parametrize("chunk", [0, 1024])
def test_tree_reduce_scatter_matches_relabelled_oracle(P, chunk):
    rc = [64 * (P - 1) * 2 + 5] * P  # permute_remap needs equal blocks
    for dtype in ("float", "int32"):
        sb = O.inputs(dtype, sum(rc), P)
        want = relabelled_rs_oracle(sb, rc, dtype)
        got = plan_sim.run("reduce_scatter", "bine_permute_remap", sb, dtype, rcounts=rc, chunk_bytes=chunk,
                           trees=True)
        for r in range(P):
            assert np.array_equal(got[r], want[r]), (P, dtype, r)
        ref, _ = O.reduce_scatter("bine_permute_remap", sb, rc, dtype)
        if dtype == "int32":
            assert all(np.array_equal(g, w) for g, w in zip(got, ref))
        else:
            assert max(float(np.max(np.abs(g - w))) for g, w in zip(got, ref)) <= P * 1e-4
        for r in range(P):
            ops, cj, fw = pico_amd.schedule("reduce_scatter", "bine_permute_remap", P, r, rcounts=rc, esz=4,
                                            chunk_bytes=chunk, trees=True)
            check_race_free(ops, cj, fw, False)
            assert len({p["peer"] for o in ops if o["xchg"] for p in o["prims"]}) == P - 1
