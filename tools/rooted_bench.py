#!/usr/bin/env python3
"""Timing of the data-movement widening (bandwidth bcasts, gather, scatter,
alltoall) in P processes sharing the box's ONE GPU over the direct
peer-memory transport, literal schedule and direct form (flat_ag), with the
HBM roofline of that one GPU: every byte a message carries is read at its
source, written into the receiver's inbox, read there and written to its
destination (4 bytes of HBM traffic per byte sent), a local block copy costs
2; the bytes of all P processes go through the one HBM (8 TB/s peak).  The
numbers say how close the schedules run to the shared HBM, NOT what xGMI
gives on a node.  Every output is checked against the collective.
usage: python tools/rooted_bench.py P [MiB per rank]   (prints one JSON line per case on rank 0)
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

HBM_PEAK = 8e12


def flat_bytes(coll, P, B):
    """HBM bytes of one call of the direct form over all ranks; B = bytes per
    block (gather / scatter / alltoall) or of the whole buffer (bcast)"""
    if coll in ("gather", "scatter"):
        return (P - 1) * B * 4 + 2 * B
    if coll == "alltoall":
        return P * ((P - 1) * B * 4 + 2 * B)
    return None   # bcasts: scatter + allgather schedules, no closed form here


def worker(rank, P, mib, port, q):
    os.environ["NCCL_HOSTID"] = f"bine-fake-host-{rank}"
    os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")
    os.environ.setdefault("NCCL_IB_DISABLE", "1")
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(P))
    import numpy as np
    import pico_amd
    import torch
    import torch.distributed as dist
    import rooted_util as R
    from oracle import oracle as O
    torch.cuda.set_device(0)
    dist.init_process_group("gloo")
    comm = pico_amd.Comm.from_torch_distributed(0)
    comm.set_direct(True)
    comm.set_chunk(64 << 20)
    stream = torch.cuda.Stream()
    per = mib << 20
    out = []
    cases = [(c, f) for c in R.ROOTED for f in (False, True)] + \
            [(("bcast", a), f) for a in ("scatter_allgather", "bine_bdw_remap") for f in (False, True)]
    for coll, flat in cases:
        comm.set_flat_ag(flat)
        if isinstance(coll, tuple):   # bcast: the whole buffer
            name, algo = coll
            n = per // 4
            buf = torch.empty(n, dtype=torch.float32, device="cuda:0")
            pico_amd.fill_pico(buf, n, "float", 77)   # the same on every rank: the result is the input
            want = buf.clone()

            def call():
                pico_amd.bcast(algo, buf, n, "float", 0, comm, stream=stream)
            got = lambda: buf
            B = per
        else:
            name, algo = coll, "bine"
            n = per // 4 // (1 if coll == "gather" else P)   # elements per block
            B = n * 4
            sb_np = R.inputs(coll, "float", n, P, seed_base=9)
            want_np, st = R.expect(coll, sb_np, "float", 0, P, n)
            assert st == 0
            s = torch.from_numpy(sb_np[rank]).to("cuda:0") if (coll != "scatter" or rank == 0) else None
            rn = {"gather": P * n if rank == 0 else 0, "scatter": n, "alltoall": P * n}[coll]
            r = torch.zeros(rn, dtype=torch.float32, device="cuda:0") if rn else None

            def call():
                if coll == "gather":
                    pico_amd.gather("bine", s, r, n, "float", 0, comm, stream=stream)
                elif coll == "scatter":
                    pico_amd.scatter("bine", s, r, n, "float", 0, comm, stream=stream)
                else:
                    pico_amd.alltoall("bine", s, r, n, "float", comm, stream=stream)
            got = lambda: r
            want = None if want_np[rank] is None else torch.from_numpy(np.ascontiguousarray(want_np[rank]))
        for _ in range(2):
            call()
        stream.synchronize()
        K = 10
        dist.barrier()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(K):
            call()
        e1.record(stream)
        stream.synchronize()
        ms = e0.elapsed_time(e1) / K
        t = torch.tensor([ms], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        ok = want is None or bool(torch.equal(got().cpu(), want.cpu()))
        okt = torch.tensor([1 if ok else 0])
        dist.all_reduce(okt, op=dist.ReduceOp.MIN)
        hb = flat_bytes(name, P, B) if flat else None
        rec = {"coll": name if isinstance(coll, str) else f"bcast_{algo}", "form": "direct" if flat else "literal",
               "P": P, "MiB_per_rank": mib, "ms": round(float(t), 4), "ok": bool(okt.item())}
        if hb:
            rec["hbm_bytes_model"] = hb
            rec["TB_s"] = round(hb / (float(t) * 1e-3) / 1e12, 3)
            rec["frac_of_8TBs"] = round(hb / (float(t) * 1e-3) / HBM_PEAK, 3)
        out.append(rec)
    if rank == 0:
        for rec in out:
            print(json.dumps(rec), flush=True)
    comm.destroy()
    dist.destroy_process_group()
    q.put((rank, all(r["ok"] for r in out)))


if __name__ == "__main__":
    import multiprocessing as mp
    import socket
    from tools._procs import join_ranks
    P = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    mib = int(sys.argv[2]) if len(sys.argv) > 2 else 64
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=worker, args=(r, P, mib, port, q)) for r in range(P)]
    for p in ps:
        p.start()
    join_ranks(ps, 280)
    res = [q.get() for _ in range(sum(1 for p in ps if p.exitcode == 0))]
    print("RESULT P=%d" % P, sorted(res), "exitcodes", [p.exitcode for p in ps], flush=True)
    sys.exit(0 if len(res) == P and all(ok for _, ok in res) else 1)
