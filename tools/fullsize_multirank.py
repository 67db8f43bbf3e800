#!/usr/bin/env python3
"""BASELINE configs C3, C4 and C5 at their FULL sizes in P = 8 real processes
(until now only the loopback transport checked them at
P = 8 in the GPU suite).  The 8 processes share the box's one GPU (distinct
NCCL_HOSTIDs); the transports are the ones bench.py picks from on the
driver's 8-GPU node: the bit-exact flat phases over the direct peer-memory
transport (flatrs+flat+dm; +dmt: its reduce-scatter trees inside the
exchange launches), the literal Bine schedule over it (direct+dm),
and the flat phases over RCCL P2P (flatrs+flat; RCCL's socket transport
here).  Inputs are pico_core's distribution generated on the device (seed
1234 + rank, exactly bench.py's); every rank's output digest is compared with
the committed oracle digest (tests/golden/bench_digests.json).
  C3: allreduce_bine_bdw_remap fp32, 256 MiB per rank
  C4: reduce_scatter_bine_permute_remap fp32, 1 GiB input per rank
  C5: allreduce_bine_bdw_remap fp64 and int64, 256 MiB per rank
usage: python tools/fullsize_multirank.py [P]   (exit 0 = every rank, every case ok)
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

CASES = [("C3", "allreduce", "bine_bdw_remap", "float", 67_108_864),
         ("C4", "reduce_scatter", "bine_permute_remap", "float", 268_435_456),
         ("C5", "allreduce", "bine_bdw_remap", "double", 33_554_432),
         ("C5", "allreduce", "bine_bdw_remap", "int64", 33_554_432)]
# (transport, which configs)
TRANSPORTS = [("flatrs+flat+dm", ("C3", "C4", "C5")), ("flatrs+flat+dmt", ("C3", "C4", "C5")),
              ("direct+dm", ("C3", "C4", "C5")), ("flatrs+flat", ("C3", "C4"))]


def worker(rank, P, port, gold, q):
    from tools._procs import rank_device
    dev = rank_device(rank)   # (sets the fake RCCL host id on the one-GPU box)
    os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")
    os.environ.setdefault("NCCL_IB_DISABLE", "1")
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(P))
    import torch
    import torch.distributed as dist
    import pico_amd
    import bench
    torch.cuda.set_device(dev)
    dist.init_process_group("gloo")
    comm = pico_amd.Comm.from_torch_distributed(dev)
    st = torch.cuda.Stream()
    tdt = {"float": torch.float32, "double": torch.float64, "int64": torch.int64}
    bad = []
    for mode, which in TRANSPORTS:
        bench.apply_transport(comm, mode, 16 << 20)
        for cfg, coll, algo, dt, n in CASES:
            if cfg not in which:
                continue
            key = f"{cfg}/{coll}/{algo}/{dt}/N{n}/P{P}"
            sb = torch.empty(n, dtype=tdt[dt], device="cuda")
            pico_amd.fill_pico(sb, n, dt, 1234 + rank)
            on = n if coll == "allreduce" else n // P
            rb = torch.empty(on, dtype=tdt[dt], device="cuda")
            rb.fill_(float("nan") if dt != "int64" else -1)
            torch.cuda.synchronize()
            dist.barrier()
            t0 = time.time()
            with torch.cuda.stream(st):
                if coll == "allreduce":
                    pico_amd.allreduce(algo, sb, rb, n, dt, "sum", comm, stream=st)
                else:
                    pico_amd.reduce_scatter(algo, sb, rb, [n // P] * P, dt, "sum", comm, stream=st)
            st.synchronize()
            comm.synchronize()
            dt_ms = (time.time() - t0) * 1e3
            d = pico_amd.checksum(rb, on, dt)
            ok = key in gold and d == int(gold[key][rank])
            if not ok:
                bad.append(f"{mode} {key}")
            print(f"rank {rank} {mode} {key}: {'ok' if ok else 'MISMATCH'} ({dt_ms:.0f} ms)", flush=True)
            del sb, rb
            torch.cuda.empty_cache()
    comm.destroy()
    dist.destroy_process_group()
    q.put((rank, len(bad)))


if __name__ == "__main__":
    import multiprocessing as mp
    from tools._procs import join_ranks
    P = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    with open(os.path.join(ROOT, "tests", "golden", "bench_digests.json")) as f:
        gold = json.load(f)["digests"]
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=worker, args=(r, P, port, gold, q)) for r in range(P)]
    for p in ps:
        p.start()
    join_ranks(ps, 900)
    res = {}
    while not q.empty():
        r, nbad = q.get()
        res[r] = nbad
    ok = len(res) == P and all(v == 0 for v in res.values()) and all(p.exitcode == 0 for p in ps)
    print(f"RESULT P={P}: {'ok' if ok else 'FAILED'} {res}", flush=True)
    sys.exit(0 if ok else 1)
