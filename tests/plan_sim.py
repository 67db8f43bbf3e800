"""Host simulator of the product's per-rank plans (test infrastructure).

Executes the primitive lists that libbine_amd.so's planner emits for ALL ranks
of a communicator, with RCCL's rendezvous semantics: the sends and receives of
one exchange group are posted together, a transfer happens when the head send
and the head receive of a (src, dst) pair are both posted, the group completes
when all its transfers did, and a rank cannot post its next group before the
current one completed.  A receive whose matching send carries a different
element count is an error (RCCL needs equal counts).  No progress while some
rank is unfinished = deadlock.  The element arithmetic of REDUCE / REDUCE3 is
MPICH's (oracle.reduce_local), so results are comparable bit-for-bit with the
oracle's restatement of the reference.
"""
from __future__ import annotations

import collections

import numpy as np

import pico_amd
from oracle import oracle as O

SB, RB, T0, T1, T2 = range(5)


class PlanError(AssertionError):
    pass


def scheduled_prims(coll, algo, P, r, chunk_bytes, relay=0, trees=False, flat_ag=False, flat_rs=False, **kw):
    """The executor's issue schedule (pico_amd.schedule) flattened back into a
    primitive list in issue order, one exchange group per op."""
    ops, _, _, info = pico_amd.schedule(coll, algo, P, r, chunk_bytes=chunk_bytes, relay_min_bytes=relay,
                                        info=True, trees=trees, flat_ag=flat_ag, flat_rs=flat_rs, **kw)
    out = []
    for i, o in enumerate(ops):
        for p in o["prims"]:
            q = dict(p)
            q["group"] = i
            out.append(q)
    return out, info


def poison(a):
    """a recognisable non-value for the device copies the staging must fill"""
    if a.dtype.kind == "f":
        a[:] = np.nan
    elif a.dtype.kind == "O":   # symbolic runs: an unwritten element is None
        a[:] = None
    else:
        a.view(np.uint8)[:] = 0xA5
    return a


def run(coll, algo, sbufs, dtype, op="sum", rcounts=None, root=0, segsize=0, in_place=False,
        rbufs=None, chunk_bytes=None, relay=0, trees=False, flat_ag=False, flat_rs=False, stage=False):
    """chunk_bytes != None: run the executor's chunked issue schedule instead of
    the plan itself (same semantics when ops run in issue order).
    stage=True (allreduce / reduce_scatter, chunk_bytes given): host staging
    (pico_amd.stage_plan) -- the device input buffer starts poisoned and is
    filled from the host input only by the h2d pieces, each applied just before
    the op it belongs to; the result returned is the HOST output, assembled only
    from the d2h pieces, each copied right after its op completed."""
    P = len(sbufs)
    esz = np.dtype(O.NP_DTYPES[dtype]).itemsize
    blocks = coll in ("gather", "scatter", "alltoall")
    if coll != "scatter":
        count = sbufs[0].size
    if coll == "scatter":   # only the root's sbuf (P blocks) is read
        count = sbufs[root].size // P
    elif coll == "alltoall":
        count = sbufs[0].size // P
    plans, bufs, stg, host_in, host_out = [], [], [], [], []
    for r in range(P):
        prims, tmp = pico_amd.plan(coll, algo, P, r, count=count, rcounts=rcounts, root=root, esz=esz,
                                   segsize=segsize, in_place=in_place)
        if chunk_bytes is not None:
            prims, info = scheduled_prims(coll, algo, P, r, chunk_bytes, relay=relay, trees=trees, flat_ag=flat_ag,
                                          flat_rs=flat_rs,
                                          count=count, rcounts=rcounts, root=root,
                                    esz=esz, segsize=segsize, in_place=in_place)
        plans.append(prims)
        if stage:
            stg.append(pico_amd.stage_plan(coll, algo, P, r, count=count, rcounts=rcounts, esz=esz,
                                           segsize=segsize, in_place=in_place, chunk_bytes=chunk_bytes,
                                           flat_ag=flat_ag, flat_rs=flat_rs))
        if blocks:
            # gather: rbuf on the root only; scatter: sbuf on the root only
            sb = sbufs[r].copy() if sbufs[r] is not None else np.zeros(0, O.NP_DTYPES[dtype])
            rn = {"gather": P * count if r == root else 0, "scatter": count, "alltoall": P * count}[coll]
            rb = poison(np.empty(rn, O.NP_DTYPES[dtype]))
        elif coll == "allgather":
            # in place: rbufs[r] already holds the rank's block where the
            # algorithm expects it (P * count elements)
            rb = np.array(rbufs[r]).copy() if in_place else poison(np.empty(P * count, O.NP_DTYPES[dtype]))
            sb = np.zeros(0, O.NP_DTYPES[dtype]) if in_place else sbufs[r].copy()
        elif rbufs is not None:
            rb = rbufs[r]
        elif coll == "reduce_scatter":   # output buffers start poisoned too (the GPU tests' NaN fill)
            rb = poison(np.empty(max(rcounts[r], 1), O.NP_DTYPES[dtype]))
        else:
            rb = poison(np.empty(max(count, 1), O.NP_DTYPES[dtype]))
        if coll != "allgather" and not blocks:
            sb = sbufs[r].copy()
        if in_place and coll != "allgather":
            if coll == "reduce_scatter":
                rb = sbufs[r].copy()
            else:
                rb = sbufs[r].copy()
            sb = rb
        if chunk_bytes is not None:
            tmp = info["tmp_elems"]  # the schedule's own plan (multi-tree plans differ)
        # workspaces start poisoned: the device's persist across calls, so a plan that
        # reads a temporary before writing it would see a previous call's bytes
        tbufs = [poison(np.empty(max(int(t), 1) + 16, O.NP_DTYPES[dtype])) for t in tmp]
        # relay staging (BINE_BUF_STAGE), exactly as large as the executor allocates
        tbufs.append(poison(np.empty(info["stage_elems"] if chunk_bytes is not None else 0, O.NP_DTYPES[dtype])))
        bufs.append([sb, rb] + tbufs)
        if stage:
            dev_in = rb if in_place else sb
            host_in.append(dev_in.copy())
            poison(dev_in)
            if not in_place:
                poison(rb)
            host_out.append(poison(rb.copy()))
    pc = [0] * P
    sendq = collections.defaultdict(collections.deque)  # (src, dst) -> [(rank, idx)]
    recvq = collections.defaultdict(collections.deque)
    posted = [None] * P      # (start, end) of the currently posted group
    pending = [0] * P        # untransferred ops in the posted group

    def view(r, buf, off, n):
        b = bufs[r][buf]
        if off + n > b.size:
            raise PlanError(f"rank {r}: buffer {buf} overflow ({off}+{n} > {b.size})")
        return b[off:off + n]

    def local(r, p):
        n = p["count"]
        if p["type"] == "COPY":
            view(r, p["dst_buf"], p["dst_off"], n)[:] = view(r, p["src_buf"], p["src_off"], n).copy()
        elif p["type"] == "REDUCE":
            io = view(r, p["dst_buf"], p["dst_off"], n)
            tmp = io.copy()
            O.reduce_local(np.ascontiguousarray(view(r, p["src_buf"], p["src_off"], n)), tmp, dtype, op)
            io[:] = tmp
        elif p["type"] == "REDUCE3":
            b = view(r, p["aux_buf"], p["aux_off"], n).copy()
            O.reduce_local(np.ascontiguousarray(view(r, p["src_buf"], p["src_off"], n)), b, dtype, op)
            view(r, p["dst_buf"], p["dst_off"], n)[:] = b
        elif p["type"] == "REDUCE_TREE":
            # leaf `pos` = aux, the k-th other leaf = src + k*n; level by level
            # v[i] = v[i] (op) v[i+w], left operand = inout (MPI_Reduce_local(in=v[i+w], inout=v[i]))
            nl, pos = p["peer"], p["pos"]
            others = iter(range(nl - 1))
            v = [view(r, p["aux_buf"], p["aux_off"], n).copy() if j == pos else
                 view(r, p["src_buf"], p["src_off"] + next(others) * n, n).copy() for j in range(nl)]
            w, lvl, swap = 1, 0, p["flags"] >> 8
            while w < nl:
                for i in range(0, nl, 2 * w):
                    if (swap >> lvl) & 1:  # v[i+w] is the inout side
                        t = v[i + w].copy()
                        O.reduce_local(np.ascontiguousarray(v[i]), t, dtype, op)
                        v[i] = t
                    else:
                        O.reduce_local(np.ascontiguousarray(v[i + w]), v[i], dtype, op)
                w *= 2
                lvl += 1
            view(r, p["dst_buf"], p["dst_off"], n)[:] = v[0]

    started = [set() for _ in range(P)]

    def begin(r, g):  # op g of rank r is about to run: its h2d pieces land first
        if stage and g not in started[r]:
            started[r].add(g)
            dev_in = bufs[r][RB if in_place else SB]
            for lo, hi in stg[r][0].get(g, []):
                dev_in[lo:hi] = host_in[r][lo:hi]

    def finish(r, old_pc):  # ops between old_pc and pc[r] are complete: their d2h pieces
        if not stage:
            return
        for j in range(old_pc, pc[r]):
            g = plans[r][j]["group"]
            last = j + 1 >= len(plans[r]) or plans[r][j + 1]["group"] != g
            if last:
                for lo, hi in stg[r][1].get(g, []):
                    host_out[r][lo:hi] = bufs[r][RB][lo:hi]

    def try_transfer(key):
        moved = False
        while sendq[key] and recvq[key]:
            (sr, si), (rr, ri) = sendq[key][0], recvq[key][0]
            s, rv = plans[sr][si], plans[rr][ri]
            if s["count"] != rv["count"]:
                raise PlanError(f"{key}: send {s['count']} vs recv {rv['count']}")
            # the executor chunks PIPELINE exchanges on both sides: the flag must
            # be symmetric or the chunk sizes of the two ends would not match
            if (s["flags"] & 1) != (rv["flags"] & 1):
                raise PlanError(f"{key}: pipelined on one side only")
            data = view(sr, s["src_buf"], s["src_off"], s["count"]).copy()
            view(rr, rv["dst_buf"], rv["dst_off"], rv["count"])[:] = data
            sendq[key].popleft(); recvq[key].popleft()
            pending[sr] -= 1; pending[rr] -= 1
            moved = True
        return moved

    while True:
        progress = False
        for r in range(P):
            while pc[r] < len(plans[r]) and posted[r] is None:
                p = plans[r][pc[r]]
                if "group" in p:
                    begin(r, p["group"])
                if p["type"] in ("SEND", "RECV"):
                    j = pc[r]
                    while j < len(plans[r]) and plans[r][j]["type"] in ("SEND", "RECV") and \
                            plans[r][j]["group"] == p["group"]:
                        x = plans[r][j]
                        if x["type"] == "SEND":
                            sendq[(r, x["peer"])].append((r, j))
                        else:
                            recvq[(x["peer"], r)].append((r, j))
                        j += 1
                    posted[r] = (pc[r], j)
                    pending[r] = j - pc[r]
                    progress = True
                else:
                    local(r, p)
                    pc[r] += 1
                    finish(r, pc[r] - 1)
                    progress = True
        for key in list(sendq.keys()):
            progress |= try_transfer(key)
        for r in range(P):
            if posted[r] is not None and pending[r] == 0:
                pc[r] = posted[r][1]
                finish(r, posted[r][0])
                posted[r] = None
                progress = True
        if all(pc[r] >= len(plans[r]) and posted[r] is None for r in range(P)):
            break
        if not progress:
            raise PlanError(f"deadlock: pcs={pc}")
    outs = []
    for r in range(P):
        rb = host_out[r] if stage else bufs[r][RB]
        if coll == "reduce_scatter":
            outs.append(rb[:rcounts[r]])
        elif coll in ("allgather", "alltoall") or (coll == "gather" and r == root):
            outs.append(rb[:P * count])
        elif coll == "gather":
            outs.append(rb[:0])
        else:
            outs.append(rb[:count])
    return outs
