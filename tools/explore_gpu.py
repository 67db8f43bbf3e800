#!/usr/bin/env python3
"""On-box exploration: reduce-kernel launch shapes on C2 and a D2D copy ceiling.

Prints one line per variant: unroll, maxblocks, nt, ms/launch, HBM GB/s (3*S/t).
Variants interleaved round-robin in one process (cdna_hip_programming.md 5.4 rule 24).
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import pico_amd

N = 16_777_216
dev = torch.device("cuda:0")
sets = 4
ins = [torch.empty(N, dtype=torch.float32, device=dev) for _ in range(sets)]
ios = [torch.empty(N, dtype=torch.float32, device=dev) for _ in range(sets)]
for k in range(sets):
    pico_amd.fill_pico(ins[k], N, "float", 1 + k)
    pico_amd.fill_pico(ios[k], N, "float", 100 + k)
torch.cuda.synchronize()
st = torch.cuda.current_stream()
variants = [(u, m, nt) for u in (2, 4, 8) for m in (0, 1024, 2048) for nt in (0, 1, 2, 3, 4, 5, 7)]
res = {v: [] for v in variants}
for rnd in range(5):
    for v in variants:
        pico_amd.set_reduce_tuning(*v)
        for i in range(4):
            pico_amd.reduce_local(ins[i % sets], ios[i % sets], N, "float", "sum", stream=st)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for i in range(40):
            pico_amd.reduce_local(ins[i % sets], ios[i % sets], N, "float", "sum", stream=st)
        e1.record(st)
        torch.cuda.synchronize()
        res[v].append(e0.elapsed_time(e1) / 40)
best = None
for v in variants:
    ms = sorted(res[v])[len(res[v]) // 2]
    gbs = 3 * N * 4 / (ms * 1e-3) / 1e9
    print(f"unroll={v[0]} maxblocks={v[1]} nt={v[2]} ms={ms:.4f} GB/s={gbs:.1f}", flush=True)
    if best is None or ms < best[1]:
        best = (v, ms)
print("BEST", best, 3 * N * 4 / (best[1] * 1e-3) / 1e9)
# copy ceiling (torch D2D copy of 64 MiB: 2*S bytes)
a, b = ins[0], ios[1]
for _ in range(5):
    b.copy_(a)
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record(st)
for i in range(40):
    ios[i % sets].copy_(ins[(i + 1) % sets])
e1.record(st)
torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / 40
print(f"copy64MiB ms={ms:.4f} GB/s(2S/t)={2 * N * 4 / (ms * 1e-3) / 1e9:.1f}")

# C3 step windows with the default shape (NT=1): per-launch sizes of the remap
# reduce-scatter at P=8 (128, 64, 32 MiB)
pico_amd.set_reduce_tuning(4, 0, 1)
big_a = torch.empty(1 << 26, dtype=torch.float32, device=dev)
big_b = torch.empty(1 << 26, dtype=torch.float32, device=dev)
pico_amd.fill_pico(big_a, 1 << 26, "float", 5)
pico_amd.fill_pico(big_b, 1 << 26, "float", 6)
for n in (1 << 25, 1 << 24, 1 << 23, 1 << 20, 1 << 16):
    offs = [0, n, 2 * n if 3 * n <= (1 << 26) else 0]
    for _ in range(3):
        pico_amd.reduce_local(big_a[offs[0]:], big_b[offs[0]:], n, "float", "sum", stream=st)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for i in range(20):
        o = offs[i % len(offs)]
        pico_amd.reduce_local(big_a[o:], big_b[o:], n, "float", "sum", stream=st)
    e1.record(st)
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 20
    print(f"window n={n} ({n * 4 >> 20} MiB) ms={ms:.4f} GB/s={3 * n * 4 / (ms * 1e-3) / 1e9:.1f}", flush=True)
