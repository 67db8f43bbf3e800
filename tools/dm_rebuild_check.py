#!/usr/bin/env python3
"""A call whose direct-transport wait timed out reports the error ITSELF, and
the transport is rebuilt by the next bine_comm_set_direct(1) on every rank
(executor.cpp): P processes on the one GPU; the wait limit is first set
absurdly low (BINE_DIRECT_TIMEOUT_S=1e-7, so the first exchange times out and
poisons the transport).  The FIRST call's completion (bine_comm_synchronize)
must raise BINE_ERR_INTERNAL on every rank whose wait timed out, its message
carrying the waiter's record; a rank whose waits
were all satisfied in time (its peers' data had arrived before it looked) may
complete the call, and then its output must match the oracle -- no rank
returns success with a wrong result.  At least one rank's first call fails,
every rank's second call fails (at issue, or at its completion: its peers'
launches exit at once), and bine_comm_direct_timed_out says so.  Then
with the limit back at 10 s set_direct(1) rebuilds it and C3 allreduces
(256 MiB fp32 per rank) match the committed oracle digest again -- with
per-exchange launches (16 MiB chunks) and with the one-launch k_dm_fused form
(64 MiB).
usage: python tools/dm_rebuild_check.py [P]   (exit 0 = every rank ok)"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def worker(rank, P, port, q):
    os.environ["NCCL_HOSTID"] = f"bine-fake-host-{rank}"
    os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")
    os.environ.setdefault("NCCL_IB_DISABLE", "1")
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(P))
    os.environ["BINE_DIRECT_TIMEOUT_S"] = "1e-7"
    import torch
    import torch.distributed as dist
    import pico_amd
    import bench
    torch.cuda.set_device(0)
    dist.init_process_group("gloo")
    stream = torch.cuda.Stream()
    n = bench.C3_ELEMS
    sb = torch.empty(n, dtype=torch.float32, device="cuda:0")
    rb = torch.empty(n, dtype=torch.float32, device="cuda:0")
    pico_amd.fill_pico(sb, n, "float", 1234 + rank)
    key = bench.gkey("C3", "allreduce", "bine_bdw_remap", "float", n, P)
    out = {}

    def call():
        # torch's fills run on its default stream, the collective on `stream`
        # (non-blocking: no implicit order between them) -- drain them first
        torch.cuda.synchronize()
        # the call's completion as the library reports it (bine_comm_synchronize)
        pico_amd.allreduce("bine_bdw_remap", sb, rb, n, "float", "sum", comm, stream=stream)
        comm.synchronize()

    # 16 MiB chunks: per-exchange launches; 64 MiB: the whole call as one
    # k_dm_fused launch -- both must report a dead transport
    for tag, chunk in (("", 16 << 20), ("_fused", 64 << 20)):
        # a fresh communicator per form: the wait limit is read when the
        # transport is built, and a healthy transport is not rebuilt
        os.environ["BINE_DIRECT_TIMEOUT_S"] = "1e-7"
        with bench.quiet_stdout():
            comm = pico_amd.Comm.from_torch_distributed(0)
        before = comm.fused_calls()
        bench.apply_transport(comm, "flatrs+flat+dmt", chunk)   # (re)builds with the tiny limit
        errs, first_ok = [], None
        for i in range(2):   # the first call's completion reports the timeout; the second fails too
            rb.fill_(float("nan"))
            torch.cuda.synchronize()
            dist.barrier()
            if i == 0 and rank > 0:
                # rank 0 issues first and waits for data its peers send only
                # later, so its wait times out for certain (with every rank
                # issuing together, all of a call's flags may be set before
                # anybody looks)
                time.sleep(0.5)
            try:
                call()
                errs.append(None)
                if i == 0:
                    first_ok = bool(bench.check_digest(pico_amd, rb, n, "float", key, rank, stream)[0])
            except pico_amd.BineError as e:
                errs.append(str(e))
        out["first_call_error" + tag] = errs[0]
        # an error names the transport and carries the waiter's record; success only with the right result
        out["first_error_recorded" + tag] = errs[0] is not None and "timed out" in errs[0] and "waited" in errs[0]
        out["first_ok_or_error" + tag] = out["first_error_recorded" + tag] or first_ok is True
        out["second_fails" + tag] = errs[1] is not None
        out["timed_out" + tag] = comm.direct_timed_out()
        torch.cuda.synchronize()
        os.environ["BINE_DIRECT_TIMEOUT_S"] = "10"
        try:
            bench.apply_transport(comm, "flatrs+flat+dmt", chunk)   # rebuilds (collective)
            ok = not comm.direct_timed_out()
            for _ in range(3):
                rb.fill_(float("nan"))
                call()
                o, _ = bench.check_digest(pico_amd, rb, n, "float", key, rank, stream)
                ok = ok and bool(o)
            out["rebuilt_ok" + tag] = ok
            out["fused_launches" + tag] = comm.fused_calls() - before
        except pico_amd.BineError as e:
            out["rebuilt_ok" + tag] = False
            out["error" + tag] = str(e)
        torch.cuda.synchronize()
        comm.destroy()
    dist.destroy_process_group()
    q.put((rank, out))


if __name__ == "__main__":
    import multiprocessing as mp
    import socket
    from tools._procs import join_ranks
    P = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=worker, args=(r, P, port, q)) for r in range(P)]
    for p in ps:
        p.start()
    join_ranks(ps, 240)
    res = {}
    while not q.empty():
        r, o = q.get()
        res[r] = o
    ok = len(res) == P and all(o["first_ok_or_error"] and o["rebuilt_ok"] and o["first_ok_or_error_fused"]
                               and o["rebuilt_ok_fused"] and o["second_fails"] and o["second_fails_fused"]
                               and o["timed_out"] and o["timed_out_fused"] and o["fused_launches_fused"] > 0
                               for o in res.values()) \
        and any(o["first_error_recorded"] for o in res.values()) \
        and any(o["first_error_recorded_fused"] for o in res.values())
    print(f"RESULT P={P}: {'ok' if ok else 'FAILED'} {res} exitcodes {[p.exitcode for p in ps]}", flush=True)
    sys.exit(0 if ok else 1)
