#!/usr/bin/env python3
"""Host-buffer collectives with the staging pipelined into the collective
(bine_allreduce_staged / bine_reduce_scatter_staged) in P real processes
sharing the box's one GPU (distinct NCCL_HOSTIDs), over RCCL and over the
direct peer-memory transport, and ("mixed") with rank 0's buffers already on
the device (NULL host pointers) while the others' are staged.  Host buffers are page-locked (as libbine.so
registers pico_core's); the device input is NaN-poisoned before every call,
so a piece the pipeline failed to copy in shows.  Every rank's host output
is compared bit for bit with the oracle (small cases: element by element;
the C3 shape, 256 MiB fp32 per rank: bine_checksum vs the committed digest
tests/golden/bench_digests.json).
usage: python tools/staged_check.py [P] [big 0|1]   (exit 0 = every rank, every case ok)
"""
import faulthandler
import json
import os
import signal
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

# (collective, algorithm, dtype, count or block, op, chunk_bytes, in_place)
CASES = [("allreduce", "bine_bdw_remap", "float", 1_000_003, "sum", 256 << 10, False),
         ("allreduce", "bine_bdw_remap", "float", 1_000_003, "sum", 1 << 20, True),
         ("allreduce", "bine_bdw_static", "double", 300_001, "sum", 256 << 10, False),
         ("allreduce", "bine_bdw_remap_segmented", "float", 500_000, "sum", 512 << 10, False),
         ("allreduce", "ring", "float", 400_003, "sum", 256 << 10, False),
         ("allreduce", "rabenseifner", "double", 200_000, "max", 256 << 10, True),
         ("allreduce", "bine_lat", "float", 65_537, "sum", 64 << 10, False),
         ("allreduce", "bine_block_by_block_any_even", "float", 300_007, "sum", 256 << 10, False),
         ("allreduce", "bine_bdw_remap", "int64", 250_000, "sum", 256 << 10, False),
         ("reduce_scatter", "bine_permute_remap", "float", 250_000, "sum", 256 << 10, False),
         ("reduce_scatter", "bine_send_remap", "float", 100_003, "sum", 256 << 10, True),
         ("reduce_scatter", "bine_static", "double", 60_001, "sum", 256 << 10, False),
         ("reduce_scatter", "bine_block_by_block", "float", 100_000, "prod", 256 << 10, False)]
C3_N = 67_108_864


def expected(P):
    from oracle import oracle as O
    want = []
    for coll, algo, dt, n, op, _, _ in CASES:
        if coll == "allreduce":
            out, rets = O.allreduce(algo, O.inputs(dt, n, P), dt, op=op)
        else:
            rc = [n] * P
            out, rets = O.reduce_scatter(algo, O.inputs(dt, n * P, P), rc, dt, op=op)
        want.append(None if any(rets) else out)
    return want


def worker(rank, P, port, want, big, q):
    os.environ["NCCL_HOSTID"] = f"bine-fake-host-{rank}"
    os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")
    os.environ.setdefault("NCCL_IB_DISABLE", "1")
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(P))
    # a stall: every thread's Python stack on SIGUSR1 (tests/_sub.py sends it
    # before its kill) and on its own after 60 s in one case
    faulthandler.register(signal.SIGUSR1, all_threads=True)
    t0 = time.time()

    def say(msg):
        print(f"[{time.time() - t0:7.2f}s] rank {rank} {msg}", flush=True)

    import numpy as np
    import torch
    import torch.distributed as dist
    import pico_amd
    from oracle import oracle as O
    torch.cuda.set_device(0)
    dist.init_process_group("gloo")
    comm = pico_amd.Comm.from_torch_distributed(0)
    st, h2d, d2h = torch.cuda.Stream(), torch.cuda.Stream(), torch.cuda.Stream()
    tdt = {"float": torch.float32, "double": torch.float64, "int64": torch.int64}
    bad = []
    for transport in ("rccl", "direct", "mixed"):
        if transport == "direct":
            say("direct transport ... start")
            comm.set_direct(True)
            say("direct transport: set")
        for (coll, algo, dt, n, op, chunk, in_place), w in zip(CASES, want):
            if w is None:
                continue
            # mixed: rank 0's buffers already on the device (NULL host
            # pointers: nothing copied for it), the others' on the host -- the
            # same schedule on every rank
            on_dev = transport == "mixed" and rank == 0
            say(f"{transport} {coll} {algo} {dt} n={n} ... start")
            faulthandler.dump_traceback_later(60, repeat=True)
            total = n if coll == "allreduce" else n * P
            inp = O.inputs(dt, total, P)[rank]
            hs = torch.from_numpy(inp.copy()).pin_memory()
            outn = total if (coll == "allreduce" or in_place) else n
            hr = torch.empty(outn, dtype=tdt[dt]).pin_memory()
            if in_place:
                hr.copy_(hs[:outn])
            else:
                hr.fill_(-7)
            ds = torch.empty(total, dtype=tdt[dt], device="cuda:0")
            dr = torch.empty(outn, dtype=tdt[dt], device="cuda:0")
            poison = float("nan") if dt != "int64" else -1
            ds.fill_(poison)
            dr.fill_(poison)
            if on_dev:  # the input where the collective reads it: ds, or dr in place
                (dr[:outn] if in_place else ds).copy_(hs[:outn] if in_place else hs)
            torch.cuda.synchronize()
            hsrc = pico_amd.IN_PLACE if in_place else (None if on_dev else hs)
            hdst = None if on_dev else hr
            if coll == "allreduce":
                pico_amd.allreduce_staged(algo, hsrc, hdst, ds, dr, n, dt, op, comm, h2d, d2h, chunk_bytes=chunk,
                                          stream=st)
            else:
                pico_amd.reduce_scatter_staged(algo, hsrc, hdst, ds, dr, [n] * P, dt, op, comm, h2d, d2h,
                                               chunk_bytes=chunk, stream=st)
            st.synchronize()
            comm.synchronize()
            if on_dev:
                hr.copy_(dr)
            got = hr.numpy()[:n] if coll == "reduce_scatter" else hr.numpy()
            ok = np.array_equal(got, w[rank])
            if not ok:
                bad.append(f"{transport} {coll} {algo} {dt} n={n} chunk={chunk} in_place={in_place}")
            faulthandler.cancel_dump_traceback_later()
            say(f"{transport} {coll} {algo} {dt} n={n} chunk={chunk >> 10}KiB in_place={in_place}: "
                f"{'ok' if ok else 'MISMATCH'}")
        if big and transport != "mixed":  # C3's shape through the staged path, vs the committed oracle digest
            with open(os.path.join(ROOT, "tests", "golden", "bench_digests.json")) as f:
                gold = json.load(f)["digests"]
            key = f"C3/allreduce/bine_bdw_remap/float/N{C3_N}/P{P}"
            say(f"{transport} C3 256 MiB staged ... start")
            faulthandler.dump_traceback_later(60, repeat=True)
            dev = torch.empty(C3_N, dtype=torch.float32, device="cuda:0")
            pico_amd.fill_pico(dev, C3_N, "float", 1234 + rank)
            hs = dev.cpu().pin_memory()
            hr = torch.empty(C3_N, dtype=torch.float32).pin_memory()
            ds = torch.full((C3_N,), float("nan"), device="cuda:0")
            dr = torch.full((C3_N,), float("nan"), device="cuda:0")
            torch.cuda.synchronize()
            pico_amd.allreduce_staged("bine_bdw_remap", hs, hr, ds, dr, C3_N, "float", "sum", comm, h2d, d2h,
                                      stream=st)
            st.synchronize()
            comm.synchronize()
            dev.copy_(hr)
            dig = pico_amd.checksum(dev, C3_N, "float")
            ok = key in gold and dig == int(gold[key][rank])
            if not ok:
                bad.append(f"{transport} C3 256 MiB")
            faulthandler.cancel_dump_traceback_later()
            say(f"{transport} C3 256 MiB staged: {'ok' if ok else 'MISMATCH'}")
    say("destroy")
    comm.destroy()
    dist.destroy_process_group()
    q.put((rank, len(bad)))


if __name__ == "__main__":
    import multiprocessing as mp
    from tools._procs import join_ranks
    faulthandler.register(signal.SIGUSR1, all_threads=True)
    P = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    big = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    want = expected(P)
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=worker, args=(r, P, port, want, big, q)) for r in range(P)]
    for p in ps:
        p.start()
    join_ranks(ps, 600)
    res = {}
    while not q.empty():
        r, nbad = q.get()
        res[r] = nbad
    ok = len(res) == P and all(v == 0 for v in res.values()) and all(p.exitcode == 0 for p in ps)
    print(f"RESULT P={P}: {'ok' if ok else 'FAILED'} {res}", flush=True)
    sys.exit(0 if ok else 1)
