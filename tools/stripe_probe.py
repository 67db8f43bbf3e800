#!/usr/bin/env python3
"""A/B of striped exchanges (bine_comm_set_stripes) and of what the split
communicators leave behind: P processes on the one GPU of the test box (RCCL
socket transport), C3 allreduce (256 MiB/rank fp32, flatrs+flat, 16 MiB
chunks), per-iteration max over ranks, median: baseline, stripes 2, stripes 4,
baseline again after the children are destroyed (set_stripes(1)), each
parity-checked.  usage: python tools/stripe_probe.py [P] [mode]
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def worker(rank, P, mode, port, q):
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
    n = bench.C3_ELEMS
    sb = torch.empty(n, dtype=torch.float32, device="cuda:0")
    rb = torch.empty(n, dtype=torch.float32, device="cuda:0")
    pico_amd.fill_pico(sb, n, "float", 1234 + rank)
    torch.cuda.synchronize()
    out = []
    for k in (1, 1, 2, 4, 1, 1, 2, 1):
        bench.apply_transport(comm, mode, 16 << 20, False, k)
        rb.fill_(float("nan"))
        st = bench.timed(torch, stream,
                         lambda: pico_amd.allreduce("bine_bdw_remap", sb, rb, n, "float", "sum", comm, stream=stream),
                         6, 2, dist, (comm.synchronize,))
        ok, _ = bench.check_digest(pico_amd, rb, n, "float",
                                   bench.gkey("C3", "allreduce", "bine_bdw_remap", "float", n, P), rank)
        out.append({"stripes": k, "ms": round(st["median_ms"], 2), "parity_ok": bench.all_ok(torch, dist, ok)})
    comm.destroy()
    dist.destroy_process_group()
    q.put((rank, out))


if __name__ == "__main__":
    import multiprocessing as mp
    P = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    mode = sys.argv[2] if len(sys.argv) > 2 else "flatrs+flat"
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=worker, args=(r, P, mode, 29631, q)) for r in range(P)]
    for p in ps:
        p.start()
    for p in ps:
        p.join(300)
    res = dict(q.get() for _ in range(sum(1 for p in ps if p.exitcode == 0)))
    print(json.dumps({"P": P, "mode": mode, "rank0": res.get(0), "exitcodes": [p.exitcode for p in ps]}), flush=True)
