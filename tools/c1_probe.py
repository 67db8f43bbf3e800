#!/usr/bin/env python3
"""C1 shape on the GPU path: allreduce fp32 1 MiB per rank (the reference's own
CPU configuration, BASELINE.md section 2: libbine bine_bdw_remap_over 381.9 us
at P = 4 through pico_core), P real processes over RCCL (on the one-GPU test
box: distinct NCCL_HOSTIDs, RCCL's socket transport -- latency figures say
nothing about xGMI).  Per algorithm x transport: per-iteration events,
median after dropping the first 20 %, host issue time per call, and parity vs
the committed oracle digests.  Meant to run under
  rocprofv3 --kernel-trace --marker-trace --stats -- python3 tools/c1_probe.py 4
with BINE_ROCTX=1, so the trace shows each step's kernel time and the host's
issue ranges (profiles/r2_c1_*).
usage: python tools/c1_probe.py [P] [iters] [MODE,MODE...]   (default: direct,flatrs+flat,direct+dm,flatrs+flat+dm)
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def worker(rank, P, iters, port, q, modes=("direct", "flatrs+flat", "direct+dm", "flatrs+flat+dm")):
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
    n = bench.C1_ELEMS
    sb = torch.empty(n, dtype=torch.float32, device="cuda:0")
    rb = torch.empty(n, dtype=torch.float32, device="cuda:0")
    pico_amd.fill_pico(sb, n, "float", 1234 + rank)
    stream = torch.cuda.current_stream()
    res = {}
    # +dm: the direct peer-memory transport; with the flat phases a C1 call is
    # then ONE k_dm_fused launch (BINE_DIRECT_FUSED=0: the primitives one by one)
    for mode in modes:
        bench.apply_transport(comm, mode, 0)
        for algo in ("bine_bdw_remap", "bine_lat"):
            st = bench.timed(torch, stream,
                             lambda: pico_amd.allreduce(algo, sb, rb, n, "float", "sum", comm, stream=stream),
                             iters, 20, dist, (comm.synchronize,))
            ok, _ = bench.check_digest(pico_amd, rb, n, "float",
                                       bench.gkey("C1", "allreduce", algo, "float", n, P), rank)
            res[f"{algo}/{mode}"] = {"us_median": round(st["median_ms"] * 1e3, 2),
                                     "host_issue_us": round(st["issue_ms"] * 1e3, 2),
                                     "parity_ok": bench.all_ok(torch, dist, ok)}
    comm.destroy()
    dist.destroy_process_group()
    q.put((rank, res))


if __name__ == "__main__":
    import multiprocessing as mp
    P = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    iters = int(sys.argv[2]) if len(sys.argv) > 2 else 200
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    modes = tuple(sys.argv[3].split(",")) if len(sys.argv) > 3 else ("direct", "flatrs+flat", "direct+dm", "flatrs+flat+dm")
    ps = [ctx.Process(target=worker, args=(r, P, iters, 29601, q, modes)) for r in range(P)]
    for p in ps:
        p.start()
    for p in ps:
        p.join(300)
    res = dict(q.get() for _ in range(sum(1 for p in ps if p.exitcode == 0)))
    print(json.dumps({"P": P, "iters": iters, "rank0": res.get(0), "exitcodes": [p.exitcode for p in ps]}), flush=True)
    sys.exit(0 if len(res) == P and all(v["parity_ok"] is not False for v in res[0].values()) else 1)
