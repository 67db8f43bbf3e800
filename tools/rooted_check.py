#!/usr/bin/env python3
"""gather_bine / scatter_bine / alltoall_bine in P real processes sharing the
box's GPU (distinct RCCL host ids): over RCCL point-to-point and over the
direct peer-memory transport, literal schedule and direct form (flat_ag),
graph mode on and off, fp32 / int64 / int8 blocks of a few sizes, root 0 and
P / 2 -- every output bit-exact vs the collective (the reference delivers it
at these (P, root), tests/rooted_util.py); the root-only buffers are None
elsewhere, as pico_core passes them.
usage: python tools/rooted_check.py [P]   (exit 0 = every rank, every case ok)
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

MODES = [("rccl", False, False, False), ("rccl", True, False, False), ("rccl", False, False, True),
         ("dm", False, True, False), ("dm", True, True, False)]   # (name, flat, direct, graphs)


def worker(rank, P, port, q):
    from tools._procs import rank_device
    dev = rank_device(rank)   # (sets the fake RCCL host id on the one-GPU box)
    os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")
    os.environ.setdefault("NCCL_IB_DISABLE", "1")
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(P))
    import numpy as np
    import pico_amd
    import torch
    import torch.distributed as dist
    import rooted_util as R
    from oracle import oracle as O
    torch.cuda.set_device(dev)
    dist.init_process_group("gloo")
    comm = pico_amd.Comm.from_torch_distributed(dev)
    stream = torch.cuda.Stream()
    bad, n_ok = [], 0
    for name, flat, direct, graphs in MODES:
        comm.set_direct(direct)
        comm.set_flat_ag(flat)
        comm.set_graphs(graphs)
        for coll in R.ROOTED:
            for dt, n in (("float", 65537), ("int64", 3), ("int8", 1 << 20)):
                for root in ([0] if coll == "alltoall" else sorted({0, P // 2})):
                    sb = R.inputs(coll, dt, n, P, seed_base=500)
                    want, exp = R.expect(coll, sb, dt, root, P, n)
                    esz = np.dtype(O.NP_DTYPES[dt]).itemsize
                    rn = {"gather": P * n if rank == root else 0, "scatter": n, "alltoall": P * n}[coll]
                    has_s = coll != "scatter" or rank == root
                    s = torch.from_numpy(sb[rank].view(np.uint8).copy()).to("cuda") if has_s else None
                    r = torch.full((rn * esz,), 0xA5, dtype=torch.uint8, device="cuda") if rn else None
                    torch.cuda.synchronize()
                    tag = f"{name} flat={flat} graphs={graphs} {coll} {dt} n={n} root={root}"
                    try:
                        for _ in range(2):   # graph mode: the second call replays
                            if coll == "gather":
                                pico_amd.gather("bine", s, r, n, dt, root, comm, stream=stream)
                            elif coll == "scatter":
                                pico_amd.scatter("bine", s, r, n, dt, root, comm, stream=stream)
                            else:
                                pico_amd.alltoall("bine", s, r, n, dt, comm, stream=stream)
                        stream.synchronize()
                        comm.synchronize()
                        got = r.cpu().numpy().view(O.NP_DTYPES[dt]) if rn else np.zeros(0, O.NP_DTYPES[dt])
                        w = want[rank]
                        ok = exp == 0 and O.canonical(got) == (b"" if w is None else O.canonical(w))
                    except pico_amd.BineError as e:
                        ok, tag = False, tag + f" error {e}"
                    if ok:
                        n_ok += 1
                    else:
                        bad.append(tag)
    for b in bad:
        print(f"rank {rank} MISMATCH {b}", flush=True)
    print(f"rank {rank}: {n_ok} ok, {len(bad)} bad", flush=True)
    comm.destroy()
    dist.destroy_process_group()
    q.put((rank, n_ok, len(bad)))


if __name__ == "__main__":
    import multiprocessing as mp
    import socket
    from tools._procs import join_ranks
    P = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=worker, args=(r, P, port, q)) for r in range(P)]
    for p in ps:
        p.start()
    join_ranks(ps, 240)
    res = [q.get() for _ in range(sum(1 for p in ps if p.exitcode == 0))]
    print("RESULT P=%d" % P, sorted(res), "exitcodes", [p.exitcode for p in ps], flush=True)
    sys.exit(0 if len(res) == P and all(b == 0 for _, _, b in res) else 1)
