"""Node model of the reduce-family collectives: what a
C3 / C4 / C5 call should take at P ranks on one node for each transport,
derived from the executed issue schedule, so the driver's first multi-GPU
line can be judged on arrival (bench.py puts `model_ms` and `frac_of_model`
in its N > 1 roofline).  Host only.

    t_model = max(t_link, t_hbm) + launches x t_boundary

* t_link: exchange ops run one after another, the links of one op in
  parallel; per op its busiest directed link's bytes at LINK_GBS (153 GB/s,
  the task's per-link figure; bench.py's link roofline uses the same sum).
* t_hbm: the HBM bytes one rank's call moves (`hbm_bytes`) at the transport
  kernels' rate.  A send reads its source (its write lands in the receiver's
  HBM and is counted there, as the receiver's arrival); a receive is that
  arrival plus -- unless a fused tree reads it in place in the inbox slot --
  the copy out of the slot / RCCL's FIFO (read + write); a tree reads its
  leaves and writes its output; a copy reads and writes; a pairwise reduction
  reads two operands and writes one.  RCCL P2P moves bytes the way the
  unfused direct transport does (FIFO in the receiver, copied out by the
  receiving kernel).
* launches: kernel launches per call (an exchange of r slot rounds: r
  launches when r = 1, else r + 1; a local op one; a fused tree none, or one
  when it is hosted by itself) x the measured launch-to-launch gap.  Over
  the direct transport with fused trees a flat call whose chunks fit (round
  5, bine_plan_dm_fused) is ONE k_dm_fused launch (a reduce-scatter: one
  per 4 chunks), whose allgather pushes come from registers.

On one GPU (P processes sharing it, the only multi-rank setting this pool
offers) every rank's bytes go through the one HBM and no link is involved:
t = P x hbm_bytes / rate + launches x t_boundary.
"""
from __future__ import annotations

LINK_GBS = 153.0          # one xGMI link, one direction (task statement); 7 per GPU
HBM_RATE_GBS = 6000.0     # the direct transport's kernels on one MI355X: 5.1-6.3 TB/s at P = 2
T_BOUNDARY_US = 7.0       # launch-to-launch gap at the default workgroups (tools/dm_stamps.py "gap_us_med",
                          # profiles/r4_dm_stamps_p2_sweep2.txt: 6.6-7.7 us)
SLOT_BYTES = 64 << 20     # the direct transport's sub-message slot (BINE_DIRECT_SLOT_BYTES)

TRANSPORTS = {
    # the transports bench.py trials (their names; "+dm16", "+dmt64x128" ...
    # are the same transports with other workgroup counts)
    "direct": "the literal Bine schedule over RCCL P2P",
    "flat": "the flat allgather phase over RCCL P2P",
    "relay": "permutation steps relayed over all links, RCCL P2P",
    "relay+flat": "relay + the flat allgather phase, RCCL P2P",
    "flatrs+flat": "flat reduce-scatter + flat allgather phases over RCCL P2P",
    "trees": "P - 1 relabelled instances on edge-disjoint pairings, RCCL P2P",
    "flatrs+flat+dm": "flat phases over the direct transport, pull copies + tree launches",
    "flatrs+flat+dmt": "flat phases over the direct transport, fused trees",
}
RELAY_MIN_BYTES = 256 << 10   # bench.py's relay setting


def _flags(transport):
    """(flat_ag, flat_rs, relay, trees, direct, fused) of a transport name"""
    t = transport
    return ("flat" in t, "flatrs" in t, "relay" in t, t.startswith("trees"), "+dm" in t, "+dmt" in t)


def _schedule(coll, algo, P, rank, esz, transport, chunk_bytes, count=0, rcounts=None):
    import pico_amd
    flat_ag, flat_rs, relay, trees, _, _ = _flags(transport)
    kw = dict(esz=esz, chunk_bytes=chunk_bytes, flat_ag=flat_ag, flat_rs=flat_rs)
    if coll == "allreduce":
        kw["count"] = count
    else:
        kw["rcounts"] = rcounts
    ops = pico_amd.schedule(coll, algo, P, rank, relay_min_bytes=RELAY_MIN_BYTES if relay and P >= 3 else 0,
                            trees=trees, **kw)[0]
    return ops, kw


def _fused(coll, algo, P, rank, kw, slot):
    """exchange ops whose receives a fused tree reads in place, the tree ops
    hosted by an exchange launch and those hosted by themselves (executor.cpp
    plan_dm_trees, via bine_plan_dm_trees)"""
    import pico_amd
    ops = pico_amd.schedule(coll, algo, P, rank, **kw)[0]
    host, _ = pico_amd.dm_tree_plan(coll, algo, P, rank, slot=slot, **kw)
    leaf_ops, self_hosted, hosted = set(), set(), set()
    for j, h in enumerate(host):
        if h < 0:
            continue
        hosted.add(j)
        if h == j:
            self_hosted.add(j)
        i = j - 1
        while not ops[i]["xchg"]:
            i -= 1
        leaf_ops.add(i)
    return leaf_ops, hosted, self_hosted


def fused_launches(coll, algo, P, rank=0, esz=4, transport="flatrs+flat+dmt", chunk_bytes=16 << 20, count=0,
                   rcounts=None, slot=SLOT_BYTES, one_launch=True):
    """k_dm_fused launches of one large call (bine_plan_dm_fused): the whole
    flat collective in one kernel (or one per 4 chunks of a reduce-scatter);
    0 = the per-exchange launches (one_launch=False: BINE_DIRECT_FUSED_LARGE=0)"""
    if not one_launch or not _flags(transport)[5] or P < 2:
        return 0
    import pico_amd
    flat_ag, flat_rs = _flags(transport)[:2]
    dt = {4: "float", 8: "double"}.get(esz, "float")
    return pico_amd.dm_fused_plan(coll, algo, P, rank, count=count, rcounts=rcounts, esz=esz, chunk_bytes=chunk_bytes,
                                  flat_ag=flat_ag, flat_rs=flat_rs, slot=slot, dtype=dt)


def hbm_bytes(coll, algo, P, rank=0, esz=4, transport="flatrs+flat+dmt", chunk_bytes=16 << 20, count=0,
              rcounts=None, slot=SLOT_BYTES, one_launch=True):
    """HBM bytes (reads + writes) one rank moves in one call (module doc).
    In the one-launch form (fused_launches > 0) every exchange that feeds a
    tree is read in place, and the allgather's sends are the trees' results
    pushed from registers: no read of their source."""
    ops, kw = _schedule(coll, algo, P, rank, esz, transport, chunk_bytes, count, rcounts)
    one = fused_launches(coll, algo, P, rank, esz, transport, chunk_bytes, count, rcounts, slot, one_launch) > 0
    if one:
        leaf_ops = {i for i in range(len(ops) - 1) if ops[i]["xchg"] and not ops[i + 1]["xchg"]}
        ag_op = len(ops) - 1 if ops and ops[-1]["xchg"] else -1
    else:
        leaf_ops = _fused(coll, algo, P, rank, kw, slot)[0] if _flags(transport)[5] else set()
        ag_op = -1
    b = 0
    for i, o in enumerate(ops):
        for p in o["prims"]:
            n = p["count"] * esz
            b += {"SEND": 0 if i == ag_op else n, "RECV": n + (0 if i in leaf_ops else 2 * n),
                  "REDUCE_TREE": (p["peer"] + 1) * n, "COPY": 2 * n, "REDUCE": 3 * n, "REDUCE3": 3 * n}[p["type"]]
    return b


def link_bytes(coll, algo, P, rank=0, esz=4, transport="flatrs+flat+dmt", chunk_bytes=16 << 20, count=0,
               rcounts=None):
    """sum over exchange ops of the busiest directed link's bytes"""
    ops, _ = _schedule(coll, algo, P, rank, esz, transport, chunk_bytes, count, rcounts)
    L = 0
    for o in ops:
        if o["xchg"]:
            lk = {}
            for p in o["prims"]:
                lk[(p["type"], p["peer"])] = lk.get((p["type"], p["peer"]), 0) + esz * p["count"]
            L += max(lk.values())
    return L


def launches(coll, algo, P, rank=0, esz=4, transport="flatrs+flat+dmt", chunk_bytes=16 << 20, count=0,
             rcounts=None, slot=SLOT_BYTES, one_launch=True):
    """kernel launches per call (module doc)"""
    nf = fused_launches(coll, algo, P, rank, esz, transport, chunk_bytes, count, rcounts, slot, one_launch)
    if nf:
        return nf
    ops, kw = _schedule(coll, algo, P, rank, esz, transport, chunk_bytes, count, rcounts)
    direct, fused = _flags(transport)[4:]
    hosted, self_hosted = (_fused(coll, algo, P, rank, kw, slot)[1:] if fused else (set(), set()))
    n = 0
    for j, o in enumerate(ops):
        if o["xchg"]:
            if direct:
                r = max(1, -(-max(p["count"] * esz for p in o["prims"]) // slot))
                n += r if r == 1 else r + 1
            else:
                n += 1
        elif j in self_hosted or j not in hosted:
            n += 1
    return n


def model_ms(coll, algo, P, esz=4, transport="flatrs+flat+dmt", chunk_bytes=16 << 20, count=0, rcounts=None,
             one_gpu=False, hbm_rate_gbs=HBM_RATE_GBS, link_gbs=LINK_GBS, t_boundary_us=T_BOUNDARY_US,
             slot=SLOT_BYTES, one_launch=True):
    """expected ms of one call (module doc): {"model_ms", "t_link_ms", "t_hbm_ms", "launches", "hbm_bytes",
    "link_bytes"} (rank 0's schedule; the collectives are symmetric)"""
    kw = dict(esz=esz, transport=transport, chunk_bytes=chunk_bytes, count=count, rcounts=rcounts)
    hb = hbm_bytes(coll, algo, P, slot=slot, one_launch=one_launch, **kw)
    lb = link_bytes(coll, algo, P, **kw) if P > 1 else 0
    nl = launches(coll, algo, P, slot=slot, one_launch=one_launch, **kw)
    t_hbm = (P if one_gpu else 1) * hb / (hbm_rate_gbs * 1e9) * 1e3
    t_link = 0.0 if one_gpu else lb / (link_gbs * 1e9) * 1e3
    return {"model_ms": round(max(t_link, t_hbm) + nl * t_boundary_us * 1e-3, 4), "t_link_ms": round(t_link, 4),
            "t_hbm_ms": round(t_hbm, 4), "launches": nl, "hbm_bytes": hb, "link_bytes": lb}


CONFIGS = {
    # BASELINE configs at full size: (collective, algorithm, element size, count or per-rank block)
    "C3": ("allreduce", "bine_bdw_remap", 4, 67_108_864),
    "C4": ("reduce_scatter", "bine_permute_remap", 4, 268_435_456),
    "C5": ("allreduce", "bine_bdw_remap", 8, 33_554_432),
}


def config_model(cfg, P, transport, chunk_bytes=16 << 20, **kw):
    coll, algo, esz, n = CONFIGS[cfg]
    if coll == "allreduce":
        return model_ms(coll, algo, P, esz=esz, transport=transport, chunk_bytes=chunk_bytes, count=n, **kw)
    return model_ms(coll, algo, P, esz=esz, transport=transport, chunk_bytes=chunk_bytes, rcounts=[n // P] * P,
                    **kw)


# ---- C1 end to end through the unchanged pico_core ----------
# pico_core hands libbine host (malloc) buffers (pico_core_allreduce_utils.c:13-25):
# a C1 call's kernels read the input and write the result in the page-locked
# host buffers over PCIe (libbine.so zero copy, round 6), every rank on its
# own GPU and its own PCIe link on a node.
T_HOST_RT_US = 54.0      # C1 at P = 1 through pico_core + libbine.so: the 1 MiB host round trip, the
                         # kernel reading and writing the page-locked host buffers over PCIe itself
                         # (round 6 zero copy; profiles/r6_e2e_c1_zero_copy.txt; staged through device
                         # buffers: 66 us, profiles/r4_e2e_c1.txt)
T_FLAG_US = 3.0          # the flag latency one k_dm_fused phase boundary costs: a system-scope store seen
                         # by the peer's poll, one way.  Assumed; bench.py measures it at N > 1
                         # (bine_comm_direct_ping: round trip / 2, "direct_transport_probe") and
                         # recomputes the models with it ("model_with_measured_constants")
C1_PHASES = 3            # k_dm_fused's flat allreduce: pushes, tree (+ allgather pushes), pulls
C1_ONE_GPU_DEV_US = {2: 28.7, 4: 49.0}   # device-resident C1 with the ranks sharing ONE GPU (one HW queue
                                          # each; profiles/r4_c1_fused_wgs.txt): the bench rehearsal's
                                          # upper bound for a node
C1_REFERENCE_CPU_US = {4: 215.0}         # the real reference libbine on the GPU box's host cores, C1 at
                                          # P = 4 (BENCH_r04 cpu_baseline)


def c1_e2e_us(P, t_host_rt_us=T_HOST_RT_US, t_flag_us=T_FLAG_US, t_boundary_us=T_BOUNDARY_US,
              link_gbs=LINK_GBS):
    """predicted C1 (fp32 allreduce_bine_bdw_remap, 262,144 elements per rank)
    end to end at P ranks of one node, one GPU + one PCIe link each, over the
    direct transport's one-launch flat form: {"e2e_us", "device_us",
    "device_us_one_gpu_bound"}.  device = one launch + C1_PHASES flag round
    trips + the busiest link's bytes; P = 1 is the measured host round trip
    alone (the collective is the copy sbuf -> rbuf)."""
    if P == 1:
        return {"e2e_us": t_host_rt_us, "device_us": 0.0, "device_us_one_gpu_bound": None}
    lb = link_bytes("allreduce", "bine_bdw_remap", P, transport="flatrs+flat+dmt", count=262_144,
                    chunk_bytes=64 << 20)
    dev = t_boundary_us + C1_PHASES * t_flag_us + lb / (link_gbs * 1e3)
    return {"e2e_us": round(t_host_rt_us + dev, 2), "device_us": round(dev, 2),
            "device_us_one_gpu_bound": C1_ONE_GPU_DEV_US.get(P)}
