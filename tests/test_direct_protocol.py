"""The direct peer-memory transport's flag protocol (pico_amd/csrc/direct.cpp)
over the executor's real issue schedules, on the host (tests/dm_sim.py):
no deadlock and no flag that moves backwards, for every transport mode the
bench trials, P = 2..8, consecutive collectives, including exchanges cut
into several slot-sized rounds and launches that carry several messages to
one peer (relay mode)."""
import pytest

import dm_sim

MODES = {
    "direct": {},
    "flat": dict(flat_ag=True),
    "flatrs+flat": dict(flat_ag=True, flat_rs=True),
    "relay": dict(relay_min_bytes=256 << 10),
    "relay+flat": dict(relay_min_bytes=256 << 10, flat_ag=True),
    "trees": dict(trees=True),
}


@pytest.mark.parametrize("P", [2, 4, 8])
@pytest.mark.parametrize("mode", sorted(MODES))
def test_allreduce_protocol_completes(P, mode):
    kw = dict(MODES[mode])
    if mode == "trees" and P not in (4, 8):
        pytest.skip("multi-tree mode: P = 4 or 8")
    res = dm_sim.run("allreduce", "bine_bdw_remap", P, count=1 << 20, chunk_bytes=1 << 20, **kw)
    assert res is None, res["stuck"][:8]


@pytest.mark.parametrize("merge", [3, 2, 1, 0])
@pytest.mark.parametrize("mode", ["direct", "relay", "flatrs+flat"])
def test_multi_round_exchanges(mode, merge):
    # slot much smaller than the messages: every exchange runs several rounds
    # and every slot is reused many times per collective; every launch
    # structure: one launch per round (2), round k-1's pulls with round k's
    # pushes (1), separate launches (0), the default mix (3)
    res = dm_sim.run("allreduce", "bine_bdw_remap", 4, count=1 << 20, chunk_bytes=4 << 20, slot=64 << 10,
                     merge=merge, **MODES[mode])
    assert res is None, res["stuck"][:8]


def test_reduce_scatter_protocol_completes():
    res = dm_sim.run("reduce_scatter", "bine_send_remap", 8, rcounts=[1 << 16] * 8, flat_rs=True)
    assert res is None, res["stuck"][:8]


@pytest.mark.parametrize("P", [2, 4, 8, 16])
@pytest.mark.parametrize("chunk", [1 << 20, 4 << 20])
def test_fused_trees_protocol_completes(P, chunk):
    # the flat reduce-scatter's trees fused into exchange launches
    # (executor.cpp plan_dm_trees): leaf pulls deferred into the next
    # exchange's first launch
    st = {}
    res = dm_sim.run("allreduce", "bine_bdw_remap", P, count=P << 20, chunk_bytes=chunk, flat_ag=2, flat_rs=True,
                     slot=1 << 20, dm_trees=True, stats=st)
    assert res is None, res["stuck"][:8]
    # leaves of several slots (chunk > slot), or P = 16 (15 deferred leaves +
    # 15 sends + 15 receives exceed one launch's 32 messages): every tree
    # runs inside its own exchange instead
    assert (st["deferred"] if P <= 8 and chunk <= 1 << 20 else st["in_exchange"]) > 0, st


@pytest.mark.parametrize("merge", [3, 2, 1, 0])
def test_fused_trees_multi_round(merge):
    # leaves of several slot rounds: trees inside their own exchange, round
    # r's tree beside round r + 1's pushes
    st = {}
    res = dm_sim.run("reduce_scatter", "bine_permute_remap", 4, rcounts=[1 << 20] * 4, chunk_bytes=4 << 20,
                     flat_rs=True, slot=256 << 10, merge=merge, dm_trees=True, stats=st)
    assert res is None, res["stuck"][:8]
    assert st["in_exchange"] > 0, st


@pytest.mark.parametrize("case", [
    ("allreduce", "bine_bdw_remap", 2, dict(count=2 << 20, chunk_bytes=1 << 20)),
    ("allreduce", "bine_bdw_remap", 4, dict(count=4 << 20, chunk_bytes=1 << 20)),
    ("allreduce", "bine_bdw_remap", 8, dict(count=8 << 20, chunk_bytes=1 << 20)),
    ("allreduce", "bine_bdw_remap", 8, dict(count=8 << 20, chunk_bytes=4 << 20)),
    ("allreduce", "bine_bdw_remap", 16, dict(count=16 << 20, chunk_bytes=1 << 20)),
    ("allreduce", "bine_bdw_static", 8, dict(count=8 << 20, chunk_bytes=1 << 20)),
    ("allreduce", "bine_bdw_remap", 8, dict(count=1_000_003, chunk_bytes=1 << 20)),
    ("allreduce", "bine_bdw_remap", 4, dict(count=4 << 20, chunk_bytes=1 << 20, in_place=True)),
    ("allreduce", "rabenseifner", 8, dict(count=8 << 20, chunk_bytes=1 << 20)),
    ("reduce_scatter", "bine_permute_remap", 8, dict(rcounts=[1 << 20] * 8, chunk_bytes=1 << 20)),
    ("reduce_scatter", "bine_send_remap", 4, dict(rcounts=[1 << 20] * 4, chunk_bytes=4 << 20)),
    ("reduce_scatter", "bine_static", 8, dict(rcounts=[1 << 20] * 8, chunk_bytes=1 << 20)),
], ids=lambda c: f"{c[0]}-{c[1]}-P{c[2]}-" + "-".join(f"{k}{v if not isinstance(v, list) else len(v)}"
                                                         for k, v in c[3].items()))
def test_simulator_restates_the_executors_tree_plan(case):
    # the simulator's dm_tree_plan (what the deadlock check runs) makes the
    # executor's plan_dm_trees decisions (bine_plan_dm_trees), rank by rank
    import pico_amd
    coll, algo, P, kw = case
    slot = 1 << 20
    n_fused = 0
    for r in range(P):
        sk = dict(kw)
        ops, _, _ = pico_amd.schedule(coll, algo, P, r, esz=4, flat_ag=2, flat_rs=True, **sk)
        host, defer = pico_amd.dm_tree_plan(coll, algo, P, r, esz=4, flat_ag=2, flat_rs=True, slot=slot, **sk)
        h, _, d = dm_sim.dm_tree_plan(ops, 4, slot)
        assert {j: x for j, x in enumerate(host) if x >= 0} == h, (r, host, h)
        assert {i for i, x in enumerate(defer) if x} == d, (r, defer, d)
        n_fused += len(h)
    assert n_fused > 0


def _hbm_bytes_per_rank(coll, algo, P, rank, fused, esz=4, **kw):
    """HBM bytes one rank moves in one call over the direct transport, from
    the executed issue schedule (pico_amd.model.hbm_bytes -- the node model
    bench.py prints beside its multi-GPU line): a push reads its source (its
    remote write is the receiver's arrival), a receive is an arrival into this
    rank's inbox plus -- unless a fused tree reads it in place -- a pull copy
    (read + write), a tree reads its leaves and writes its output, a copy
    reads and writes, a pairwise reduction reads two operands and writes one"""
    from pico_amd import model
    return model.hbm_bytes(coll, algo, P, rank, esz=esz, transport="flatrs+flat+dmt" if fused else "flatrs+flat+dm",
                           slot=1 << 20, **kw)


@pytest.mark.parametrize("P", [4, 8])
def test_hbm_model_of_the_fused_trees(P):
    # DESIGN.md §3 "Push groups" table: HBM bytes per rank per C3 call at P = 8,
    # unfused 8.125 S vs fused trees 6.375 S (7.25 / 5.75 S at P = 4), and the
    # reduce_scatter C4 (S = input): 4.625 / 2.875 S at P = 8
    S = (P << 20) * 4
    ar = {f: _hbm_bytes_per_rank("allreduce", "bine_bdw_remap", P, 0, f, count=P << 20, chunk_bytes=1 << 20) / S
          for f in (False, True)}
    want = {8: (8.125, 6.375), 4: (7.25, 5.75)}[P]
    assert (ar[False], ar[True]) == want, ar
    rs = {f: _hbm_bytes_per_rank("reduce_scatter", "bine_permute_remap", P, 0, f, rcounts=[1 << 20] * P,
                                 chunk_bytes=1 << 20) / S for f in (False, True)}
    if P == 8:
        assert (rs[False], rs[True]) == (4.625, 2.875), rs
    assert rs[True] < rs[False]
