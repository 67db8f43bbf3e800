#!/usr/bin/env python3
"""tools/graph_fork_repro.cpp in a torch process, i.e. on the HIP runtime torch
bundles (7.0 in this image) -- the runtime the round-3 crash happened in.  A
two-branch graph (stream A forks B, a kernel on each, A joins B) captured
with hipStreamBeginCapture through torch.cuda.graph and replayed.  Prints
"GRAPH_FORK ok" when the replays ran (libbine-free)."""
import os

import torch

s1 = torch.cuda.Stream()
s2 = torch.cuda.Stream()
x = torch.zeros(1 << 20, device="cuda")
y = torch.zeros(1 << 20, device="cuda")
torch.cuda.synchronize()
print("torch", torch.__version__, "HIP", torch.version.hip, "GPU_MAX_HW_QUEUES =",
      os.environ.get("GPU_MAX_HW_QUEUES", "(default)"), flush=True)
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g, stream=s1):
    s2.wait_stream(s1)          # fork
    with torch.cuda.stream(s2):
        y.add_(1.0)
    x.add_(2.0)
    s1.wait_stream(s2)          # join
print("captured; replaying", flush=True)
for _ in range(3):
    g.replay()
torch.cuda.synchronize()
ok = float(x[7]) == 6.0 and float(y[7]) == 3.0
print("GRAPH_FORK", "ok" if ok else "WRONG", float(x[7]), float(y[7]), flush=True)
raise SystemExit(0 if ok else 1)
