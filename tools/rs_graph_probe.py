#!/usr/bin/env python3
"""bench.py's C4 side measurement in isolation: reduce_scatter_bine_permute_remap
fp32, 1 GiB input per rank, P processes on the one GPU (distinct
NCCL_HOSTIDs), on a given transport x chunk x graph-mode setting -- the
configuration a 4-process rehearsal with GPU_MAX_HW_QUEUES=1 picked for C3
(flatrs+flat+dm16, 64 MiB chunks, graph replay) and then crashed in (host
SIGSEGV inside the C4 call).  Each rank prints before every call, runs with
Python's faulthandler and BINE_SEGV_TRACE=1 (native stack of a fatal
signal), and checks its output digest against the committed oracle digest.
usage: python tools/rs_graph_probe.py P MODE CHUNK_MIB GRAPHS(0/1) [ITERS]
"""
import faulthandler
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def worker(rank, P, mode, chunk, graphs, iters, port, q):
    faulthandler.enable()
    os.environ["NCCL_HOSTID"] = f"bine-fake-host-{rank}"
    os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")
    os.environ.setdefault("NCCL_IB_DISABLE", "1")
    os.environ.setdefault("BINE_SEGV_TRACE", "1")
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
    n = bench.C4_ELEMS
    sb = torch.empty(n, dtype=torch.float32, device="cuda:0")
    rb = torch.empty(n // P, dtype=torch.float32, device="cuda:0")
    pico_amd.fill_pico(sb, n, "float", 1234 + rank)
    bench.apply_transport(comm, mode, chunk, graphs)
    key = bench.gkey("C4", "reduce_scatter", "bine_permute_remap", "float", n, P)
    oks = []
    for it in range(iters):
        print(f"rank {rank} {mode}/{chunk >> 20}MiB graphs={graphs} call {it} ...", flush=True)
        rb.fill_(float("nan"))
        pico_amd.reduce_scatter("bine_permute_remap", sb, rb, [n // P] * P, "float", "sum", comm, stream=stream)
        torch.cuda.synchronize()
        comm.synchronize()
        ok, _ = bench.check_digest(pico_amd, rb, n // P, "float", key, rank, stream)
        oks.append(ok)
    print(f"rank {rank} done: digests {oks}", flush=True)
    comm.set_graphs(False)
    comm.destroy()
    dist.destroy_process_group()
    q.put((rank, all(o is not False for o in oks)))


if __name__ == "__main__":
    import multiprocessing as mp
    from tools._procs import join_ranks
    P, mode, chunk, graphs = int(sys.argv[1]), sys.argv[2], int(sys.argv[3]) << 20, sys.argv[4] == "1"
    iters = int(sys.argv[5]) if len(sys.argv) > 5 else 3
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=worker, args=(r, P, mode, chunk, graphs, iters, 29621, q)) for r in range(P)]
    for p in ps:
        p.start()
    join_ranks(ps, 300)
    res = [q.get() for _ in range(sum(1 for p in ps if p.exitcode == 0))]
    print("RESULT", sorted(res), "exitcodes", [p.exitcode for p in ps], flush=True)
    sys.exit(0 if len(res) == P and all(ok for _, ok in res) else 1)
