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


# ---- residency -------------------------------------------------
# The trial that timed out in two of six 8-rank rehearsals on one GPU (DESIGN.md
# section 4.4): relay+flat+dm, C3 (67,108,864 fp32 per rank), 16 MiB chunks, 64 MiB
# slots, RELAY_MIN_BYTES 256 KiB, the default 128 workgroups per message cut by
# share / 2 = 4 to 32.  k_dm_move holds 32 VGPRs (8 waves per SIMD: 8 workgroups
# of 256 threads per CU), so one MI355X has 256 x 8 = 2048 workgroup slots.
TRIAL = dict(count=67_108_864, esz=4, chunk_bytes=16 << 20, relay_min_bytes=256 << 10, flat_ag=True,
             slot=64 << 20, merge=3)
SLOTS_MI355X = 256 * 8


def test_relay_flat_dm_trial_protocol_is_deadlock_free():
    """the exact trial configuration with every workgroup resident: the
    protocol itself completes -- the recorded timeout was not a protocol
    deadlock"""
    assert dm_sim.run("allreduce", "bine_bdw_remap", 8, calls=2, **TRIAL) is None


def test_shared_gpu_residency_stall_and_the_cut():
    """8 ranks on one GPU: without the library's residency cut a dispatcher
    order exists in which the chip fills with waiting workgroups whose
    producers have no slot (a residency stall -- what the hardware scheduler
    resolves by time slicing, slowly, or not within the 10 s wait); with
    the cut (dm_fit_residency: each launch <= slots / ranks on the GPU) every
    co-located rank's current launch is resident at once and no dispatcher
    order stalls"""
    kw = dict(TRIAL, count=8 << 20)
    gpu = {"gpu_of": [0] * 8, "slots": SLOTS_MI355X}
    st = {}
    res = dm_sim.run("allreduce", "bine_bdw_remap", 8, calls=2, stats=st,
                     residency=dict(gpu, wgs=128, cap=False, policy="seq"), **kw)
    assert res is not None and res["residency"] and res["free_slots"] == [0]
    assert st["max_launch_wgs"] == 14 * 128   # 7 pushes + 7 pulls of 128 workgroups
    for pol in ("seq", "rr", "adv"):
        for wgs in (32, 128):
            st = {}
            res = dm_sim.run("allreduce", "bine_bdw_remap", 8, calls=2, stats=st,
                             residency=dict(gpu, wgs=wgs, cap=True, policy=pol), **kw)
            assert res is None, (pol, wgs, res and res["stuck"][:4])
            assert st["max_launch_wgs"] <= SLOTS_MI355X // 8 and st["max_gpu_wgs"] <= SLOTS_MI355X


def test_node_residency_one_rank_per_gpu():
    """one rank per GPU (the node): launches larger than the chip complete
    without the cut too (dispatch is in order within a launch and nothing a
    workgroup waits for sits behind it on its own GPU); the cut makes every
    launch one wave of residency"""
    kw = dict(TRIAL, count=16 << 20)
    for cap in (False, True):
        st = {}
        res = dm_sim.run("allreduce", "bine_bdw_remap", 8, calls=2, stats=st,
                         residency={"gpu_of": list(range(8)), "slots": SLOTS_MI355X, "wgs": 256, "cap": cap,
                                    "policy": "seq"}, **kw)
        assert res is None
        assert (st["max_launch_wgs"] <= SLOTS_MI355X) == cap


def test_fit_residency_library_matches_restatement():
    """bine_dm_fit_residency (the library's cut) == dm_sim.fit on random
    launches: sum <= cap, every part >= 1, unchanged when it fits"""
    import ctypes
    import random
    import pico_amd
    L = pico_amd.lib()
    rng = random.Random(5)
    for _ in range(2000):
        n = rng.randint(0, 32)
        cw = [rng.choice([1, 16, 32, 64, 128, 256, 512]) * rng.randint(1, 3) for _ in range(n)]
        tw = rng.choice([None, 0, 32, 256, 512])
        cap = rng.choice([0, 1, 8, 64, 160, 256, 1280, 2048, 4096])
        a = (ctypes.c_int * max(n, 1))(*cw)
        t = ctypes.c_int(tw or 0)
        rc = L.bine_dm_fit_residency(a, n, ctypes.byref(t) if tw is not None else None, cap)
        pc, pt = list(cw), ([tw] if tw is not None else None)
        want = dm_sim.fit(pc, pt, cap)
        assert rc == want, (cw, tw, cap)
        assert list(a)[:n] == pc and (tw is None or t.value == pt[0])
        if rc == 1:
            assert sum(pc) + (pt[0] if pt else 0) <= cap and min(pc + [1]) >= 1
        if rc == 0:
            assert pc == cw


def test_fused_residency_margin_and_slice_flags():
    """k_dm_fused with 8 ranks on one MI355X (256 CUs x 5
    resident blocks = 1,280 slots).  Round 5's cap (CUs x blocks / share =
    160 per rank) demands exactly 1,280: with whole-message flags every
    workgroup of every rank must be resident at once, so ONE slot held by any
    other wave stalls the call until a waiter times out -- the rehearsal's
    record (the producers' marks arrived after the time-out).  The bound: the
    margin (one block per CU left free: 128 per rank, 1,024 slots) completes
    with up to one held slot per CU; slice flags (a workgroup waits only for
    its peers' same slice, dispatch in blockIdx order) complete at the old
    cap with up to W - 1 held slots."""
    import pico_amd
    L = pico_amd.lib()
    cus, per = 256, 5
    assert L.bine_dm_residency_cap(cus, per, 0, 8) == 160          # round 5's rule
    assert L.bine_dm_residency_cap(cus, per, 1, 8) == 128          # the margin
    assert L.bine_dm_residency_cap(cus, per, 1, 2) == 512          # P = 2 keeps its 512 workgroups
    assert L.bine_dm_residency_cap(cus, per, 1, 1) == 1024         # a node: above every default launch
    assert L.bine_dm_residency_cap(cus, 1, 1, 1) == cus            # never below one block per CU
    assert L.bine_dm_residency_cap(0, per, 1, 1) == 0               # unknown device
    for share in range(1, 17):
        for p in range(2, 9):
            for m in (0, 1, 2):
                cap = L.bine_dm_residency_cap(cus, p, m, share)
                assert cap == cus * max(1, p - m) // share
                assert share * cap <= cus * p - (cus * m if p - m >= 1 else 0)
    slots = cus * per
    for order in ("rr", "seq"):
        assert dm_sim.fused_residency(8, 160, slots, 0, slices=False, order=order) == (True, 1280)
        assert dm_sim.fused_residency(8, 160, slots, 1, slices=False, order=order) == (False, 1279)
        assert dm_sim.fused_residency(8, 128, slots, cus, slices=False, order=order) == (True, 1024)
        assert not dm_sim.fused_residency(8, 128, slots, cus + 1, slices=False, order=order)[0]
        assert dm_sim.fused_residency(8, 160, slots, 159, slices=True, order=order)[0]
        assert dm_sim.fused_residency(8, 128, slots, cus, slices=True, order=order)[0]


# ---- the one-launch form moves the per-exchange form's messages (round 5) ----------

def _per_exchange_msgs(ops, esz, slot, rank_peer_kind):
    """the per-exchange launches' messages of one rank in sequence order, per
    (peer, push): each exchange's message to / from a peer cut into slot-sized
    rounds (DirectState::exchange), exchanges in issue order (a deferred
    tree's leaf pulls keep their place relative to the same peer's later
    receives)"""
    out = {}
    for o in ops:
        if not o["xchg"]:
            continue
        for p in o["prims"]:
            if p["type"] not in ("SEND", "RECV") or not p["count"]:
                continue
            b = p["count"] * esz
            key = (p["peer"], 1 if p["type"] == "SEND" else 0)
            k = 0
            while k * slot < b:
                out.setdefault(key, []).append(min(slot, b - k * slot))
                k += 1
    return out


FUSED_CASES = [
    # (coll, algo, P, count or block, esz, chunk, slot, ragged)
    ("allreduce", "bine_bdw_remap", 2, 67_108_864, 4, 64 << 20, 64 << 20, False),
    ("allreduce", "bine_bdw_remap", 4, 67_108_864, 4, 64 << 20, 64 << 20, False),
    ("allreduce", "bine_bdw_remap", 8, 67_108_864, 4, 64 << 20, 64 << 20, False),
    ("allreduce", "bine_bdw_remap", 8, 33_554_432, 8, 64 << 20, 64 << 20, False),
    ("allreduce", "bine_bdw_remap", 2, 2 * (262_144 + 64), 4, 1 << 20, 1 << 20, False),      # a short last chunk
    ("allreduce", "bine_bdw_remap", 4, 4 * (262_144 + 4), 4, 1 << 20, 1 << 20, False),
    ("allreduce", "bine_bdw_static", 8, 8 * 262_144 * 2, 4, 1 << 20, 1 << 20, False),
    ("allreduce", "rabenseifner", 4, 4 * (131_072 + 2), 8, 1 << 20, 1 << 20, False),
    ("reduce_scatter", "bine_permute_remap", 2, 6 * 262_144, 4, 1 << 20, 1 << 20, False),
    ("reduce_scatter", "bine_permute_remap", 8, 268_435_456 // 8, 4, 64 << 20, 64 << 20, False),
    ("reduce_scatter", "bine_send_remap", 4, 3 * 262_144, 4, 1 << 20, 1 << 20, True),
]


@pytest.mark.parametrize("case", FUSED_CASES, ids=lambda c: f"{c[0]}-{c[1]}-P{c[2]}-n{c[3]}")
def test_one_launch_form_moves_the_per_exchange_messages(case):
    """bine_plan_dm_fused_msgs vs the per-exchange form: for every rank and
    peer the one-launch program pushes (and pulls) the same message sizes in
    the same order as the per-exchange launches, and rank x's pushes to y are
    rank y's pulls from x -- so every pair of ranks agrees on every sequence
    number whichever form each rank takes (executor.cpp plan_fused)"""
    import pico_amd
    coll, algo, P, n, esz, chunk, slot, ragged = case
    dt = {4: "float", 8: "double"}[esz]
    kw = dict(esz=esz, chunk_bytes=chunk, flat_ag=coll == "allreduce", flat_rs=True)
    if coll == "allreduce":
        kw["count"] = n
    else:
        kw["rcounts"] = [n + (4 * (r % 3) if ragged else 0) for r in range(P)]   # ragged, 16-B blocks
    seqs, n_fused = {}, 0
    for r in range(P):
        nl, msgs = pico_amd.dm_fused_msgs(coll, algo, P, r, slot=slot, dtype=dt, **kw)
        ops = pico_amd.schedule(coll, algo, P, r, **kw)[0]
        per = _per_exchange_msgs(ops, esz, slot, None)
        seqs[r] = per
        if nl == 0:
            continue   # this rank keeps the per-exchange launches (e.g. ragged: a send-only last exchange)
        n_fused += 1
        got = {}
        for _, push, peer, b in msgs:
            got.setdefault((peer, push), []).append(b)
        assert got == per, (case, r)
        seqs[r] = got
    assert n_fused >= 1, case
    # every ordered pair agrees, whichever form each end takes
    for x in range(P):
        for y in range(P):
            if x != y:
                assert seqs[x].get((y, 1), []) == seqs[y].get((x, 0), []), (case, x, y)
