#!/usr/bin/env python3
"""Functional check of the RCCL transport with P ranks sharing ONE GPU.

RCCL refuses two ranks on one device of one host ("Duplicate GPU detected"),
so each rank claims a different host id (NCCL_HOSTID) and RCCL connects them
over its socket network transport on the loopback interface.  This validates
the executor's RCCL path (grouping, stream/event hand-offs, chunked pipeline,
exact counts) with real multi-process RCCL; it says nothing about xGMI speed.
usage: python tools/rccl_1gpu_multirank.py [P] [relay_min_bytes] [trees 0|1]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def worker(rank, P, port, q, relay=0, trees=0):
    os.environ["NCCL_HOSTID"] = f"bine-fake-host-{rank}"
    os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")
    os.environ.setdefault("NCCL_IB_DISABLE", "1")
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(P))
    import numpy as np
    import torch
    import torch.distributed as dist
    import pico_amd
    from oracle import oracle as O
    torch.cuda.set_device(0)
    dist.init_process_group("gloo")
    comm = pico_amd.Comm.from_torch_distributed(0)
    comm.set_relay(relay)
    comm.set_trees(bool(trees))
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    ok = True
    for algo, n, seg in (("bine_bdw_remap", 100003, 0), ("bine_bdw_remap", 100003, 4096),
                         ("bine_bdw_static", 4099, 0), ("ring", 4099, 0), ("bine_lat", 333, 0),
                         ("bine_bdw_remap_segmented", 5000, 64), ("bine_block_by_block_any_even", 4099, 0)):
        sb = O.inputs("float", n, P)
        if trees and P in (4, 8) and n >= 64 * (P - 1):
            import test_trees
            want = test_trees.relabelled_oracle(algo, sb, "float", segsize=seg)
        else:
            want, _ = O.allreduce(algo, sb, "float", segsize=seg)
        s = torch.from_numpy(sb[rank]).cuda()
        r = torch.zeros_like(s)
        pico_amd.allreduce(algo, s, r, n, "float", "sum", comm, segsize=seg)
        torch.cuda.synchronize()
        comm.synchronize()
        same = np.array_equal(r.cpu().numpy(), want[rank])
        ok &= same
        print(f"rank {rank} {algo} n={n} seg={seg} relay={relay} trees={trees}: {'ok' if same else 'MISMATCH'}", flush=True)
    rc = [4096] * P
    sb = O.inputs("float", sum(rc), P)
    want, _ = O.reduce_scatter("bine_permute_remap", sb, rc, "float")
    s = torch.from_numpy(sb[rank]).cuda()
    r = torch.zeros(rc[rank], dtype=torch.float32, device="cuda:0")
    pico_amd.reduce_scatter("bine_permute_remap", s, r, rc, "float", "sum", comm)
    torch.cuda.synchronize()
    same = np.array_equal(r.cpu().numpy(), want[rank])
    ok &= same
    print(f"rank {rank} reduce_scatter_bine_permute_remap: {'ok' if same else 'MISMATCH'}", flush=True)
    comm.destroy()
    dist.destroy_process_group()
    q.put((rank, ok))


if __name__ == "__main__":
    import multiprocessing as mp
    P = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    relay = int(sys.argv[2]) if len(sys.argv) > 2 else 0
    trees = int(sys.argv[3]) if len(sys.argv) > 3 else 0
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=worker, args=(r, P, 29555, q, relay, trees)) for r in range(P)]
    for p in ps:
        p.start()
    for p in ps:
        p.join(300)
    res = [q.get() for _ in range(sum(1 for p in ps if p.exitcode == 0))]
    print("RESULT", res, "exitcodes", [p.exitcode for p in ps])
    sys.exit(0 if len(res) == P and all(ok for _, ok in res) else 1)
