#!/usr/bin/env python3
"""The direct peer-memory transport (bine_comm_set_direct) in real processes:
P processes on the one GPU of the test box (cross-process VMM mappings of one
device; timings say nothing about xGMI), C3 allreduce (256 MiB/rank fp32) per
transport, RCCL vs direct, per-iteration max over ranks, median; parity vs the
committed oracle digests.  usage: python tools/direct_probe.py [P] [n] [modes]
(PROBE_DM_ONLY=1: the direct transport only)
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def worker(rank, P, n, modes, port, q):
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
    sb = torch.empty(n, dtype=torch.float32, device="cuda:0")
    rb = torch.empty(n, dtype=torch.float32, device="cuda:0")
    pico_amd.fill_pico(sb, n, "float", 1234 + rank)
    torch.cuda.synchronize()
    key = bench.gkey("C3" if n == bench.C3_ELEMS else "C1", "allreduce", "bine_bdw_remap", "float", n, P)
    out = {}
    for mode in modes:
        for direct in ((True,) if os.environ.get("PROBE_DM_ONLY") == "1" else (False, True)):
            bench.apply_transport(comm, mode, 16 << 20)
            comm.set_direct(direct)
            rb.fill_(float("nan"))
            try:
                st = bench.timed(torch, stream,
                                 lambda: pico_amd.allreduce("bine_bdw_remap", sb, rb, n, "float", "sum", comm,
                                                            stream=stream), 6, 2, dist, (comm.synchronize,))
                ok, _ = bench.check_digest(pico_amd, rb, n, "float", key, rank)
                out[f"{mode}{'+dm' if direct else ''}"] = {"ms": round(st["median_ms"], 3),
                                                          "parity_ok": bench.all_ok(torch, dist, ok)}
            except pico_amd.BineError as e:
                out[f"{mode}{'+dm' if direct else ''}"] = {"error": str(e)[:200]}
            print(f"rank {rank} {mode} direct={direct}: {out}", flush=True)
    comm.set_direct(False)
    comm.destroy()
    dist.destroy_process_group()
    q.put((rank, out))


if __name__ == "__main__":
    import multiprocessing as mp
    from tools._procs import join_ranks
    P = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 67_108_864
    modes = sys.argv[3].split(",") if len(sys.argv) > 3 else ["direct", "flatrs+flat"]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=worker, args=(r, P, n, modes, 29641, q)) for r in range(P)]
    for p in ps:
        p.start()
    join_ranks(ps, 300)
    for p in ps:
        if p.is_alive():
            p.kill()
    res = dict(q.get() for _ in range(sum(1 for p in ps if p.exitcode == 0)))
    print(json.dumps({"P": P, "n": n, "rank0": res.get(0), "exitcodes": [p.exitcode for p in ps]}), flush=True)
