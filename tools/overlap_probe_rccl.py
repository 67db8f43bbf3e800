#!/usr/bin/env python3
"""Recv/reduce overlap of the two-stream executor over real RCCL (VERDICT r1
item 7): P processes on the one GPU of the test box (distinct NCCL_HOSTIDs,
RCCL's socket transport), config C4 -- reduce_scatter_bine_permute_remap, fp32,
1 GiB input per rank -- and C3 (allreduce_bine_bdw_remap 256 MiB/rank) at the
default 16 MiB pipelining chunk, literal transport.  Per collective: rank 0's
per-op profile (comm-stream exchanges vs compute-stream reductions,
bench.step_profile: the share of reduction time during which an exchange is
in flight) and parity vs the committed oracle digests.  Run under
  rocprofv3 --kernel-trace --output-format csv -d DIR -- python3 tools/overlap_probe_rccl.py 4
and summarise the trace with tools/rccl_overlap_report.py DIR (RCCL kernels
vs k_reduce kernels, per process).
usage: python tools/overlap_probe_rccl.py [P] [mode]
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def worker(rank, P, mode, port, q):
    os.environ["NCCL_HOSTID"] = f"bine-fake-host-{rank}"
    os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")
    os.environ.setdefault("NCCL_IB_DISABLE", "1")
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(P))
    import torch
    import torch.distributed as dist
    import pico_amd
    import bench
    torch.cuda.set_device(0)
    dist.init_process_group("gloo")
    with bench.quiet_stdout():
        comm = pico_amd.Comm.from_torch_distributed(0)
    bench.apply_transport(comm, mode, 0)
    stream = torch.cuda.current_stream()
    out = {}
    n = bench.C4_ELEMS
    sb = torch.empty(n, dtype=torch.float32, device="cuda:0")
    rb = torch.empty(n // P, dtype=torch.float32, device="cuda:0")
    pico_amd.fill_pico(sb, n, "float", 1234 + rank)
    rc = [n // P] * P
    call = lambda: pico_amd.reduce_scatter("bine_permute_remap", sb, rb, rc, "float", "sum", comm,  # noqa: E731
                                           stream=stream)
    call()
    torch.cuda.synchronize()
    prof = bench.step_profile(torch, comm, call)
    ok, _ = bench.check_digest(pico_amd, rb, n // P, "float",
                               bench.gkey("C4", "reduce_scatter", "bine_permute_remap", "float", n, P), rank)
    out["C4"] = {k: prof[k] for k in ("ops", "span_ms", "exchange_busy_ms", "local_busy_ms", "overlap_frac")}
    out["C4"]["parity_ok"] = bench.all_ok(torch, dist, ok)
    del sb, rb
    n = bench.C3_ELEMS
    sb = torch.empty(n, dtype=torch.float32, device="cuda:0")
    rb = torch.empty(n, dtype=torch.float32, device="cuda:0")
    pico_amd.fill_pico(sb, n, "float", 1234 + rank)
    call = lambda: pico_amd.allreduce("bine_bdw_remap", sb, rb, n, "float", "sum", comm, stream=stream)  # noqa: E731
    call()
    torch.cuda.synchronize()
    prof = bench.step_profile(torch, comm, call)
    ok, _ = bench.check_digest(pico_amd, rb, n, "float",
                               bench.gkey("C3", "allreduce", "bine_bdw_remap", "float", n, P, mode == "trees"), rank)
    out["C3"] = {k: prof[k] for k in ("ops", "span_ms", "exchange_busy_ms", "local_busy_ms", "overlap_frac")}
    out["C3"]["parity_ok"] = bench.all_ok(torch, dist, ok)
    comm.destroy()
    dist.destroy_process_group()
    q.put((rank, out))


if __name__ == "__main__":
    import multiprocessing as mp
    P = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    mode = sys.argv[2] if len(sys.argv) > 2 else "direct"
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=worker, args=(r, P, mode, 29611, q)) for r in range(P)]
    for p in ps:
        p.start()
    for p in ps:
        p.join(300)
    res = dict(q.get() for _ in range(sum(1 for p in ps if p.exitcode == 0)))
    print(json.dumps({"P": P, "mode": mode, "per_rank": res, "exitcodes": [p.exitcode for p in ps]}), flush=True)
    sys.exit(0 if len(res) == P else 1)
