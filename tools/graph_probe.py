#!/usr/bin/env python3
"""Can a whole Bine collective -- RCCL P2P groups on the comm stream, reduce
kernels on the caller's stream, the event hand-offs between them -- be
captured into one HIP graph and replayed?  (round 1's
capture attempt crashed inside RCCL; this probe isolates it.)

P processes on the one GPU of the test box (distinct NCCL_HOSTIDs: RCCL's
socket transport).  Per case: one eager call (builds the plan, the schedule
and the workspace -- nothing may allocate during capture), then capture of ONE
call with torch.cuda.graph on a side stream, then replays; every replay's
output digest vs the oracle's (tests/golden/bench_digests.json, C1 inputs),
and per-call time eager vs replayed.
usage: python tools/graph_probe.py [P] [capture_error_mode | lib] [elements] [transports]
("lib": the library's graph mode, bine_comm_set_graphs, instead of a torch capture)
(elements > 262,144 = more than 1 MiB: the two-stream schedule; transports
comma-separated, default direct,flatrs+flat)
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def worker(rank, P, mode, port, q, n, transports):
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
    sb = torch.empty(n, dtype=torch.float32, device="cuda:0")
    rb = torch.empty(n, dtype=torch.float32, device="cuda:0")
    pico_amd.fill_pico(sb, n, "float", 1234 + rank)
    out = {}
    for transport in transports:
        bench.apply_transport(comm, transport, 0)
        for algo in ("bine_bdw_remap", "bine_lat"):
            tag = f"{algo}/{transport}"
            key = bench.gkey("C1" if n == bench.C1_ELEMS else "C3", "allreduce", algo, "float", n, P)
            s = torch.cuda.Stream()
            res = {}
            try:
                with torch.cuda.stream(s):
                    pico_amd.allreduce(algo, sb, rb, n, "float", "sum", comm, stream=s)
                torch.cuda.synchronize()
                comm.synchronize()
                dist.barrier()
                reps = 50 if n <= bench.C1_ELEMS else 5
                t0 = time.perf_counter()
                for _ in range(reps):
                    pico_amd.allreduce(algo, sb, rb, n, "float", "sum", comm, stream=s)
                torch.cuda.synchronize()
                comm.synchronize()
                res["eager_us"] = round((time.perf_counter() - t0) / reps * 1e6, 1)
                dist.barrier()
                if mode == "lib":   # the library's own graph mode (bine_comm_set_graphs)
                    comm.set_graphs(True)
                    pico_amd.allreduce(algo, sb, rb, n, "float", "sum", comm, stream=s)   # eager + capture

                    class _G:
                        @staticmethod
                        def replay():
                            pico_amd.allreduce(algo, sb, rb, n, "float", "sum", comm, stream=s)
                    g = _G()
                else:
                    g = torch.cuda.CUDAGraph()
                    with torch.cuda.graph(g, stream=s, capture_error_mode=mode):
                        print(f"rank {rank} {tag}: capturing", flush=True)
                        pico_amd.allreduce(algo, sb, rb, n, "float", "sum", comm, stream=s)
                res["captured"] = True
                dist.barrier()
                ok = True
                for i in range(3):
                    rb.fill_(float("nan"))
                    torch.cuda.synchronize()
                    g.replay()
                    torch.cuda.synchronize()
                    comm.synchronize()
                    o, _ = bench.check_digest(pico_amd, rb, n, "float", key, rank)
                    ok = ok and bool(o)
                res["replay_parity_ok"] = bench.all_ok(torch, dist, ok)
                dist.barrier()
                t0 = time.perf_counter()
                for _ in range(reps):
                    g.replay()
                torch.cuda.synchronize()
                res["replay_us"] = round((time.perf_counter() - t0) / reps * 1e6, 1)
                del g
                comm.set_graphs(False)
            except Exception as e:  # noqa: BLE001 -- reported
                res["error"] = f"{type(e).__name__}: {e}"[:300]
                torch.cuda.synchronize()
            out[tag] = res
            print(f"rank {rank} {tag}: {res}", flush=True)
    comm.destroy()
    dist.destroy_process_group()
    q.put((rank, out))


if __name__ == "__main__":
    import multiprocessing as mp
    P = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    mode = sys.argv[2] if len(sys.argv) > 2 else "thread_local"
    n = int(sys.argv[3]) if len(sys.argv) > 3 else 262_144
    transports = sys.argv[4].split(",") if len(sys.argv) > 4 else ["direct", "flatrs+flat"]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=worker, args=(r, P, mode, 29621, q, n, transports)) for r in range(P)]
    for p in ps:
        p.start()
    for p in ps:
        p.join(240)
    for p in ps:
        if p.is_alive():
            p.kill()
    res = dict(q.get() for _ in range(sum(1 for p in ps if p.exitcode == 0)))
    print(json.dumps({"P": P, "mode": mode, "rank0": res.get(0), "exitcodes": [p.exitcode for p in ps]}), flush=True)
