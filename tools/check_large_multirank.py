#!/usr/bin/env python3
"""On-box check of large collectives with P ranks sharing ONE GPU (fake RCCL
host ids): event time vs host wall time per call, and the result of a slice
against a gloo all_reduce of the same inputs.  Diagnoses timing artefacts.
usage: torchrun --nproc-per-node P tools/check_large_multirank.py
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
rank = int(os.environ["RANK"])
os.environ["NCCL_HOSTID"] = f"bine-fake-host-{rank}"
os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")
import torch
import torch.distributed as dist
import pico_amd

P = int(os.environ["WORLD_SIZE"])
torch.cuda.set_device(0)
dist.init_process_group("gloo")
comm = pico_amd.Comm.from_torch_distributed(0)
st = torch.cuda.current_stream()
for dt, tdt, n in (("float", torch.float32, 1 << 22), ("double", torch.float64, 33_554_432),
                   ("float", torch.float32, 67_108_864)):
    sb = torch.empty(n, dtype=tdt, device="cuda:0")
    rb = torch.empty(n, dtype=tdt, device="cuda:0")
    pico_amd.fill_pico(sb, n, dt, 5 + rank)
    for relay in (0, 262144):
        comm.set_relay(relay)
        pico_amd.allreduce("bine_bdw_remap", sb, rb, n, dt, "sum", comm, stream=st)
        torch.cuda.synchronize(); comm.synchronize(); dist.barrier()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        e0.record(st)
        for _ in range(5):
            pico_amd.allreduce("bine_bdw_remap", sb, rb, n, dt, "sum", comm, stream=st)
        e1.record(st)
        torch.cuda.synchronize(); comm.synchronize()
        wall = (time.perf_counter() - t0) / 5 * 1e3
        ev = e0.elapsed_time(e1) / 5
        sl = sb[: 1 << 20].cpu()
        dist.all_reduce(sl)
        got = rb[: 1 << 20].cpu()
        err = float((got - sl).abs().max())
        tail = rb[-(1 << 20):].cpu()
        tl = sb[-(1 << 20):].cpu()
        dist.all_reduce(tl)
        err = max(err, float((tail - tl).abs().max()))
        if rank == 0:
            print(f"{dt} n={n} ({n * sb.element_size() >> 20} MiB) relay={relay}: event {ev:.3f} ms  "
                  f"wall {wall:.3f} ms  max|err| {err:.3g}", flush=True)
    del sb, rb
    torch.cuda.empty_cache()
comm.destroy()
dist.destroy_process_group()
