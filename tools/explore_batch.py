#!/usr/bin/env python3
"""On-box: one batched launch of the P-1 chunk reductions of a multi-tree round
vs one launch per window (P = 8: 7 windows; the window sizes of C3's three
reduce-scatter steps in tree mode).  HBM GB/s = 3 * bytes / t."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import pico_amd

st = torch.cuda.current_stream()
for mib in (9.14, 4.57, 2.29, 0.5):
    n = int(mib * (1 << 18)) // 16 * 16
    a = [torch.empty(n, dtype=torch.float32, device="cuda:0") for _ in range(7)]
    b = [torch.empty(n, dtype=torch.float32, device="cuda:0") for _ in range(7)]
    for k in range(7):
        pico_amd.fill_pico(a[k], n, "float", k + 1)
        pico_amd.fill_pico(b[k], n, "float", k + 11)
    res = {}
    for mode in ("batched", "separate"):
        def run():
            if mode == "batched":
                assert pico_amd.reduce_batch(a, b, [n] * 7, "float", stream=st) == 0
            else:
                for k in range(7):
                    pico_amd.reduce_local(a[k], b[k], n, "float", "sum", stream=st)
        for _ in range(3):
            run()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(50):
            run()
        e1.record(st)
        torch.cuda.synchronize()
        res[mode] = e0.elapsed_time(e1) / 50
    gb = 3 * 7 * n * 4 / 1e9
    print(f"7 x {n * 4 / 2**20:.2f} MiB: batched {res['batched'] * 1e3:.1f} us ({gb / res['batched'] * 1e3:.0f} GB/s)"
          f"  separate {res['separate'] * 1e3:.1f} us ({gb / res['separate'] * 1e3:.0f} GB/s)", flush=True)
