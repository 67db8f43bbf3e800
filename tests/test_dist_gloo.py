"""Multi-process (world_size 2, 4 and 8 -- the driver's node size --, gloo, CPU) execution of the product's
per-rank plans: every process builds ITS OWN plan with libbine_amd.so's planner
and executes it with torch.distributed point-to-point (one batch of isend /
irecv per exchange group = ncclGroupStart/End semantics), the element
arithmetic done by the oracle's MPI_Reduce_local.  Results must equal the
oracle's restatement of the reference bit-for-bit on every rank.  This is the
N > 1 path of the executor with the transport swapped for gloo."""
import os
import socket

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CASES = [
    ("allreduce", "bine_bdw_remap", "float", 1001),
    ("allreduce", "bine_bdw_static", "float", 999),
    ("allreduce", "bine_bdw_remap_segmented", "double", 777),
    ("allreduce", "bine_lat", "int64", 129),
    ("allreduce", "ring", "float", 1000),
    ("allreduce", "rabenseifner", "float", 1000),
    ("allreduce", "recursivedoubling", "int32", 65),
    ("allreduce", "bine_block_by_block_any_even", "float", 1003),
    ("reduce_scatter", "bine_permute_remap", "float", 64),
    ("reduce_scatter", "bine_send_remap", "float", 64),
    ("reduce_scatter", "bine_static", "double", 64),
    ("reduce_scatter", "bine_block_by_block", "float", 64),
    ("reduce_scatter", "bine_block_by_block_any_even", "float", 64),
    ("reduce_scatter", "ring", "float", 64),
    ("reduce_scatter", "butterfly", "float", 64),
    ("reduce_scatter", "recursivehalving", "float", 64),
    ("reduce_scatter", "recursive_distance_doubling", "float", 64),
    ("reduce", "bine_bdw", "float", 1000),
    ("reduce", "bine_lat", "float", 1000),
    ("allgather", "bine_permute_remap", "float", 100),
    ("allgather", "bine_send_static", "int8", 33),
    ("allgather", "bine_2_blocks", "float", 10),
    ("allgather", "k_bruck", "double", 7),
    ("allgather", "sparbit", "float", 5),
    ("allgather", "bine_block_by_block", "float", 9),
    # gather / scatter / alltoall (round 5): n = elements per block, root 0
    ("gather", "bine", "float", 7),
    ("scatter", "bine", "int64", 5),
    ("alltoall", "bine", "float", 3),
]
# the flat reduce-scatter + flat allgather phases (one all-peers exchange per
# phase, REDUCE_TREE on the owner), executed from the issue schedule
FLAT_CASES = [
    ("allreduce", "bine_bdw_remap", "float", 1001),
    ("allreduce", "bine_bdw_static", "double", 999),
    ("allreduce", "rabenseifner", "int64", 1000),
    ("reduce_scatter", "bine_permute_remap", "float", 64),
    ("reduce_scatter", "bine_static", "float", 64),
    ("reduce_scatter", "bine_block_by_block", "float", 64),
    ("reduce", "bine_bdw", "double", 1000),
    ("reduce", "bine_lat", "float", 1000),
    ("allreduce", "bine_lat", "double", 1000),
    ("allreduce", "recursivedoubling", "int32", 65),
    ("allreduce", "bine_block_by_block_any_even", "float", 1003),
    ("reduce_scatter", "butterfly", "float", 64),
    ("reduce_scatter", "recursive_distance_doubling", "float", 64),
    ("reduce_scatter", "bine_block_by_block_any_even", "float", 64),
    ("allreduce", "ring", "float", 1000),
    ("reduce_scatter", "ring", "double", 64),
    ("gather", "bine", "int8", 9),
    ("scatter", "bine", "float", 4),
    ("alltoall", "bine", "int64", 2),
]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, P, port, q):
    import sys
    sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
    import torch
    import torch.distributed as dist
    import pico_amd
    from oracle import oracle as O
    import rooted_util as R
    dist.init_process_group("gloo", rank=rank, world_size=P, init_method=f"tcp://127.0.0.1:{port}")
    bad = []
    for flat, (coll, algo, dtype, n) in [(False, c) for c in CASES] + [(True, c) for c in FLAT_CASES]:
        npdt = O.NP_DTYPES[dtype]
        esz = np.dtype(npdt).itemsize
        rc = [n // P] * P if coll == "reduce_scatter" else None
        total = sum(rc) if rc else n
        sb = O.inputs(dtype, total, P)
        if coll in R.ROOTED:
            sb = R.inputs(coll, dtype, n, P)
            want = R.expect(coll, sb, dtype, 0, P, n)[0][rank]
        elif coll == "allgather":
            want = O.allgather(algo, sb, dtype)[0][rank]
        elif coll == "allreduce":
            want = O.allreduce(algo, sb, dtype, segsize=64)[0][rank]
        elif coll == "reduce_scatter":
            want = O.reduce_scatter(algo, sb, rc, dtype)[0][rank]
        else:
            want = O.reduce(algo, sb, dtype)[0] if rank == 0 else None
        if not flat:
            prims, tmp = pico_amd.plan(coll, algo, P, rank, count=n, rcounts=rc, esz=esz, segsize=64)
        else:  # the executor's issue schedule, one exchange group per op
            ops, _, _, info = pico_amd.schedule(coll, algo, P, rank, count=n, rcounts=rc, esz=esz, segsize=64,
                                                chunk_bytes=128, flat_rs=True, flat_ag=True, info=True)
            prims = [dict(x, group=k) for k, o in enumerate(ops) for x in o["prims"]]
            tmp = info["tmp_elems"]
        out_n = rc[rank] if rc else (P * n if coll in ("allgather", "alltoall") or (coll == "gather" and rank == 0)
                                     else 0 if coll == "gather" else n)
        bufs = [sb[rank].copy(), np.zeros(max(out_n, 1), npdt)] + [np.zeros(int(t) + 1, npdt) for t in tmp]

        def v(b, off, cnt):
            return bufs[b][off:off + cnt]

        i = 0
        while i < len(prims):
            p = prims[i]
            if p["type"] in ("SEND", "RECV"):
                reqs, j = [], i
                while j < len(prims) and prims[j]["type"] in ("SEND", "RECV") and prims[j]["group"] == p["group"]:
                    x = prims[j]
                    if x["type"] == "SEND":
                        t = torch.from_numpy(v(x["src_buf"], x["src_off"], x["count"]).copy().view(np.uint8))
                        reqs.append(dist.isend(t, x["peer"]))
                    else:
                        t = torch.from_numpy(v(x["dst_buf"], x["dst_off"], x["count"]).view(np.uint8))
                        reqs.append(dist.irecv(t, x["peer"]))
                    j += 1
                for r in reqs:
                    r.wait()
                i = j
                continue
            cnt = p["count"]
            if p["type"] == "COPY":
                v(p["dst_buf"], p["dst_off"], cnt)[:] = v(p["src_buf"], p["src_off"], cnt).copy()
            elif p["type"] == "REDUCE_TREE":  # level by level, left = inout (bit 8+l: swapped)
                nl, pos, swap = p["peer"], p["pos"], p["flags"] >> 8
                others = iter(range(nl - 1))
                vv = [v(p["aux_buf"], p["aux_off"], cnt).copy() if j == pos else
                      v(p["src_buf"], p["src_off"] + next(others) * cnt, cnt).copy() for j in range(nl)]
                w, lvl = 1, 0
                while w < nl:
                    for k in range(0, nl, 2 * w):
                        inout, inp = (vv[k + w], vv[k]) if (swap >> lvl) & 1 else (vv[k], vv[k + w])
                        io = inout.copy()
                        O.reduce_local(np.ascontiguousarray(inp), io, dtype)
                        vv[k] = io
                    w, lvl = w * 2, lvl + 1
                v(p["dst_buf"], p["dst_off"], cnt)[:] = vv[0]
            elif p["type"] == "REDUCE":
                io = v(p["dst_buf"], p["dst_off"], cnt)
                tmpio = io.copy()
                O.reduce_local(np.ascontiguousarray(v(p["src_buf"], p["src_off"], cnt)), tmpio, dtype)
                io[:] = tmpio
            else:
                b = v(p["aux_buf"], p["aux_off"], cnt).copy()
                O.reduce_local(np.ascontiguousarray(v(p["src_buf"], p["src_off"], cnt)), b, dtype)
                v(p["dst_buf"], p["dst_off"], cnt)[:] = b
            i += 1
        if want is not None and not np.array_equal(bufs[1][:out_n], want):
            bad.append((coll, algo, "flat" if flat else "literal"))
        dist.barrier()
    dist.destroy_process_group()
    q.put((rank, bad))


@pytest.mark.parametrize("P", [2, 4, 8])
def test_plans_over_gloo(P):
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, P, port, q)) for r in range(P)]
    for p in ps:
        p.start()
    res = [q.get(timeout=300) for _ in range(P)]
    for p in ps:
        p.join(60)
    assert all(p.exitcode == 0 for p in ps)
    bad = [x for _, b in res for x in b]
    assert not bad, bad


def _stats_worker(rank, P, port, q):
    import sys
    sys.path[:0] = [ROOT]
    import torch
    import torch.distributed as dist
    import bench
    dist.init_process_group("gloo", rank=rank, world_size=P, init_method=f"tcp://127.0.0.1:{port}")
    per = [[1.0, 5.0, 3.0, 3.0, 3.0], [2.0, 1.0, 4.0, 4.0, 4.0]][rank]
    st = bench.reduce_stats(torch, dist, per, 3.0 + rank, 0.1 * (rank + 1), 1.0)
    verdicts = [bench.all_ok(torch, dist, v) for v in ([True, False][rank], [None, True][rank], None, True)]
    dist.destroy_process_group()
    q.put((rank, st, verdicts))


def test_bench_statistic_and_verdicts_over_gloo():
    """bench.py's cross-rank reduction: per-iteration max over ranks, first
    20 % dropped, median; parity verdicts: any False fails every rank, None
    (unchecked) only if no rank checked"""
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_stats_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = dict((r, (st, v)) for r, st, v in (q.get(timeout=120) for _ in range(2)))
    for p in ps:
        p.join(60)
    for r in (0, 1):
        st, v = res[r]
        # max over ranks per iteration [2, 5, 4, 4, 4] -> drop 1 -> [5, 4, 4, 4]
        assert st["median_ms"] == 4.0 and st["max_ms"] == 5.0 and st["samples"] == 4
        assert st["region_ms"] == 4.0 and abs(st["issue_ms"] - 0.2) < 1e-12
        assert v == [False, True, None, True]
