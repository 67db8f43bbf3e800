#!/usr/bin/env python3
"""What makes the one-launch form time out with 8 ranks on ONE GPU (VERDICT
r5 item 3): C3 (allreduce_bine_bdw_remap fp32, 256 MiB per
rank) over the direct transport's flat phases at 64 MiB chunks -- one
k_dm_fused launch per call -- issued the way bench.py's trials issue it
(batches of calls back to back, then a synchronize), P processes sharing the
GPU.  Per rank: the wall time of every batch, the first error (a timed-out
wait carries the waiter's record and both ends' flags and bases,
DirectState::describe), and the output digest against the committed oracle
digest.  The variables under test come from the environment of the run:
GPU_MAX_HW_QUEUES (HW queues per priority of each rank), BINE_DIRECT_TIMEOUT_S
(a starved rank that later runs completes within a longer limit; a protocol
deadlock never does), BINE_DIRECT_FUSED_WGS (workgroups per launch: the
residency margin).  Rank 0 prints one JSON line with every rank's summary and
the box's queue census.
usage: python tools/fused8_probe.py [P] [BATCHES] [CALLS_PER_BATCH]"""
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def worker(rank, P, port, batches, per, q):
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
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    n = bench.C3_ELEMS
    sb = torch.empty(n, dtype=torch.float32, device="cuda:0")
    rb = torch.empty(n, dtype=torch.float32, device="cuda:0")
    pico_amd.fill_pico(sb, n, "float", 1234 + rank)
    torch.cuda.synchronize()
    bench.apply_transport(comm, os.environ.get("PROBE_TRANSPORT", "flatrs+flat+dmt"),
                          int(os.environ.get("PROBE_CHUNK_MIB", "64")) << 20)
    key = bench.gkey("C3", "allreduce", "bine_bdw_remap", "float", n, P)
    times, err, ok, census = [], None, None, None
    fused0 = comm.fused_calls()
    for b in range(batches):
        dist.barrier()
        t0 = time.perf_counter()
        d = bench.Drain(comm)
        g = d.guard(lambda: pico_amd.allreduce("bine_bdw_remap", sb, rb, n, "float", "sum", comm, stream=stream))
        for _ in range(per):
            g()
        torch.cuda.synchronize()
        d()
        times.append((time.perf_counter() - t0) * 1e3)
        if b == 0 and rank == 0:
            census = bench.queue_census()   # every rank's queues exist by now
        why = d.failed(dist)
        if why is not None:
            err = d.err
            break
    if err is None:
        ok = bool(bench.check_digest(pico_amd, rb, n, "float", key, rank, stream)[0])
    out = {"rank": rank, "batches": len(times), "batch_ms_median": round(statistics.median(times), 3) if times else None,
           "batch_ms_max": round(max(times), 3) if times else None, "fused_launches": comm.fused_calls() - fused0,
           "digest_ok": ok, "error": err[:2500] if err else None, "census_after_batch0": census}
    comm.destroy()
    dist.destroy_process_group()
    q.put(out)


if __name__ == "__main__":
    import multiprocessing as mp
    import socket
    from tools._procs import join_ranks
    import bench
    P = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    batches = int(sys.argv[2]) if len(sys.argv) > 2 else 12
    per = int(sys.argv[3]) if len(sys.argv) > 3 else 5
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=worker, args=(r, P, port, batches, per, q)) for r in range(P)]
    for p in ps:
        p.start()
    census = None
    t0 = time.time()
    while any(p.is_alive() for p in ps) and time.time() - t0 < 8:
        time.sleep(0.5)
    census = bench.queue_census()   # while the ranks run
    join_ranks(ps, 420)
    res = []
    while not q.empty():
        res.append(q.get())
    env = {k: os.environ.get(k) for k in ("GPU_MAX_HW_QUEUES", "BINE_DIRECT_TIMEOUT_S", "BINE_DIRECT_FUSED_WGS",
                                          "PROBE_TRANSPORT", "PROBE_CHUNK_MIB", "BINE_COMM_PRIORITY")}
    ok = len(res) == P and all(r["error"] is None and r["digest_ok"] for r in res)
    print(json.dumps({"P": P, "env": env, "ok": ok, "census_while_running": census,
                      "ranks": sorted(res, key=lambda r: r["rank"])}), flush=True)
    sys.exit(0 if ok else 1)
