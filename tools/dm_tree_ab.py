#!/usr/bin/env python3
"""Trees inside the exchange vs pull copies + separate tree launches over the
direct transport (flatrs+flat+dmt / flatrs+flat+dm, i.e.
bine_comm_set_direct_tree 1 / 0), P processes on the one GPU (distinct
NCCL_HOSTIDs; GPU_MAX_HW_QUEUES as the caller sets it): C3
(allreduce_bine_bdw_remap fp32 256 MiB per rank) and C4
(reduce_scatter_bine_permute_remap fp32 1 GiB input per rank) at each chunk,
per-iteration events (bench.timed: max over ranks, median after dropping
20 %), every output digest-checked against the committed oracle digests.
One process group per setting.  On one GPU all ranks share one HBM, so the
figures rank the two forms by the HBM traffic they cause -- not an xGMI
measurement.
usage: python tools/dm_tree_ab.py P [CHUNK_MIB,...] [ITERS] [WGS]
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def worker(rank, P, tree, chunks, iters, wgs, port, q):
    os.environ["BINE_DIRECT_TREE"] = "1" if tree else "0"
    os.environ["NCCL_HOSTID"] = f"bine-fake-host-{rank}"
    os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")
    os.environ.setdefault("NCCL_IB_DISABLE", "1")
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(P))
    import torch
    import torch.distributed as dist
    import pico_amd
    import bench
    torch.cuda.set_device(0)
    dist.init_process_group("gloo")
    with bench.quiet_stdout():
        comm = pico_amd.Comm.from_torch_distributed(0)
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    res = {}
    mode = ("flatrs+flat+dmt" if tree else "flatrs+flat+dm") + (str(wgs) if wgs else "")
    for cfg, n, coll in (("C3", bench.C3_ELEMS, "allreduce"), ("C4", bench.C4_ELEMS, "reduce_scatter")):
        sb = torch.empty(n, dtype=torch.float32, device="cuda:0")
        nout = n if coll == "allreduce" else n // P
        rb = torch.empty(nout, dtype=torch.float32, device="cuda:0")
        pico_amd.fill_pico(sb, n, "float", 1234 + rank)
        for ch in chunks:
            bench.apply_transport(comm, mode, ch << 20)
            rb.fill_(float("nan"))
            if coll == "allreduce":
                fn = lambda: pico_amd.allreduce("bine_bdw_remap", sb, rb, n, "float", "sum", comm, stream=stream)
                key = bench.gkey("C3", "allreduce", "bine_bdw_remap", "float", n, P)
            else:
                fn = lambda: pico_amd.reduce_scatter("bine_permute_remap", sb, rb, [n // P] * P, "float", "sum",
                                                     comm, stream=stream)
                key = bench.gkey("C4", "reduce_scatter", "bine_permute_remap", "float", n, P)
            st = bench.timed(torch, stream, fn, iters, 3, dist, (comm.synchronize,))
            ok, _ = bench.check_digest(pico_amd, rb, nout, "float", key, rank, stream)
            res[f"{cfg}/{ch}MiB"] = {"ms": round(st["median_ms"], 4), "min_ms": round(st["min_ms"], 4),
                                    "max_ms": round(st["max_ms"], 4), "parity_ok": bench.all_ok(torch, dist, ok)}
        del sb, rb
        torch.cuda.empty_cache()
    comm.destroy()
    dist.destroy_process_group()
    q.put((rank, res))


def run(P, tree, chunks, iters, wgs, port):
    import multiprocessing as mp
    from tools._procs import join_ranks
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=worker, args=(r, P, tree, chunks, iters, wgs, port, q)) for r in range(P)]
    for p in ps:
        p.start()
    join_ranks(ps, 400)
    res = dict(q.get() for _ in range(sum(1 for p in ps if p.exitcode == 0)))
    return res.get(0), [p.exitcode for p in ps]


if __name__ == "__main__":
    P = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    chunks = [int(x) for x in sys.argv[2].split(",")] if len(sys.argv) > 2 else [16, 64]
    iters = int(sys.argv[3]) if len(sys.argv) > 3 else 10
    wgs = int(sys.argv[4]) if len(sys.argv) > 4 else 0
    out, ok = {}, True
    for tree, port in ((True, 29641), (False, 29642)):
        r0, codes = run(P, tree, chunks, iters, wgs, port)
        name = "tree_in_exchange" if tree else "pull_copies_then_tree"
        out[name] = {"rank0": r0, "exitcodes": codes}
        print(json.dumps({name: out[name]}), flush=True)
        ok = ok and r0 is not None and all(c == 0 for c in codes) and all(v["parity_ok"] is not False
                                                                          for v in r0.values())
    print(json.dumps({"P": P, "GPU_MAX_HW_QUEUES": os.environ.get("GPU_MAX_HW_QUEUES"), **out}), flush=True)
    sys.exit(0 if ok else 1)
