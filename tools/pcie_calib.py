#!/usr/bin/env python3
"""PCIe calibration of the box (the end-to-end staging's bound): 256 MiB
host<->device copies from page-locked host memory, host->device alone,
device->host alone, and both directions at once on two streams (PCIe is full
duplex), plus the same from pageable memory.  GB/s = bytes / time per
direction, median of 7.  usage: python tools/pcie_calib.py [MiB]"""
import json
import statistics
import sys

import torch

MIB = int(sys.argv[1]) if len(sys.argv) > 1 else 256
n = MIB << 20
dev = torch.device("cuda:0")
d_a = torch.empty(n, dtype=torch.uint8, device=dev)
d_b = torch.empty(n, dtype=torch.uint8, device=dev)
out = {"bytes": n}
for pinned in (True, False):
    h_a = torch.empty(n, dtype=torch.uint8, pin_memory=pinned)
    h_b = torch.empty(n, dtype=torch.uint8, pin_memory=pinned)
    h_a.fill_(1)
    s1, s2 = torch.cuda.Stream(dev), torch.cuda.Stream(dev)

    def run(h2d, d2h):
        torch.cuda.synchronize()
        e = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
        e[0].record(s1)
        e[2].record(s2)
        if h2d:
            with torch.cuda.stream(s1):
                d_a.copy_(h_a, non_blocking=True)
        if d2h:
            with torch.cuda.stream(s2):
                h_b.copy_(d_b, non_blocking=True)
        e[1].record(s1)
        e[3].record(s2)
        torch.cuda.synchronize()
        return e[0].elapsed_time(e[1]), e[2].elapsed_time(e[3])
    res = {}
    for name, a, b in (("h2d", True, False), ("d2h", False, True), ("both", True, True)):
        ts = [run(a, b) for _ in range(8)][1:]
        t1 = statistics.median(x[0] for x in ts)
        t2 = statistics.median(x[1] for x in ts)
        r = {}
        if a:
            r["h2d_GBs"] = round(n / (t1 * 1e-3) / 1e9, 2)
        if b:
            r["d2h_GBs"] = round(n / (t2 * 1e-3) / 1e9, 2)
        if a and b:
            r["both_ms"] = round(max(t1, t2), 3)
        res[name] = r
    out["pinned" if pinned else "pageable"] = res
print(json.dumps(out))
