#!/usr/bin/env python3
"""Workload for the overlap evidence: P virtual ranks (loopback) on one GPU run
allreduce_bine_bdw_remap fp32 with the default 16 MiB pipelining chunk, so a
kernel + memory-copy trace shows the exchanges of chunk k+1 (copies on the
comm streams) running while chunk k is reduced (k_reduce on the compute
streams).  usage: python tools/overlap_probe.py [P] [MiB]
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import pico_amd

P = int(sys.argv[1]) if len(sys.argv) > 1 else 2
n = (int(sys.argv[2]) if len(sys.argv) > 2 else 256) << 18
comms = pico_amd.Comm.loopback(P, 0)
sb = [torch.empty(n, dtype=torch.float32, device="cuda:0") for _ in range(P)]
rb = [torch.empty(n, dtype=torch.float32, device="cuda:0") for _ in range(P)]
for r in range(P):
    pico_amd.fill_pico(sb[r], n, "float", r + 1)
torch.cuda.synchronize()
for _ in range(4):
    rc, st = pico_amd.loopback_allreduce(comms, "bine_bdw_remap", sb, rb, n, "float")
    assert rc == 0, st
torch.cuda.synchronize()
for c in comms:
    c.destroy()
print("done", P, n)
