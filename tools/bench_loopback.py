#!/usr/bin/env python3
"""On-box timing of the executor with P virtual ranks on ONE GPU (loopback
transport: exchanges are device copies on each rank's comm stream).  All ranks
share one HBM, so absolute numbers are not xGMI numbers; what this measures is
the executor itself -- chunking, stream overlap, launch overhead -- as the
pipelining chunk varies.  Prints one line per (algo, P, chunk): ms per
collective (median of rounds) and HBM-side bytes/s of the whole job.
usage: python tools/bench_loopback.py [MiB_per_rank]
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import pico_amd

MiB = int(sys.argv[1]) if len(sys.argv) > 1 else 64
n = MiB << 18  # floats
dev = torch.device("cuda:0")
for P in (2, 4, 8):
    comms = pico_amd.Comm.loopback(P, 0)
    sb = [torch.empty(n, dtype=torch.float32, device=dev) for _ in range(P)]
    rb = [torch.empty(n, dtype=torch.float32, device=dev) for _ in range(P)]
    for r in range(P):
        pico_amd.fill_pico(sb[r], n, "float", r + 1)
    torch.cuda.synchronize()
    for algo in ("bine_bdw_remap", "bine_bdw_static", "ring"):
        for chunk in (1 << 50, 16 << 20, 4 << 20, 1 << 20):
            rc, _ = pico_amd.loopback_allreduce(comms, algo, sb, rb, n, "float", segsize=chunk)
            assert rc == 0, rc
            ts = []
            for _ in range(7):
                t0 = time.perf_counter()
                rc, _ = pico_amd.loopback_allreduce(comms, algo, sb, rb, n, "float", segsize=chunk)
                ts.append(time.perf_counter() - t0)
            ms = sorted(ts)[len(ts) // 2] * 1e3
            tag = "none" if chunk >= 1 << 40 else f"{chunk >> 20}MiB"
            print(f"P={P} {algo:18s} chunk={tag:6s} ms={ms:8.3f} algbw/rank={n * 4 / (ms * 1e-3) / 1e9:7.1f} GB/s",
                  flush=True)
    for c in comms:
        c.destroy()
    del sb, rb
    torch.cuda.empty_cache()
