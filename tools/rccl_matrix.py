#!/usr/bin/env python3
"""Every algorithm of every family through the RCCL transport, P real processes
sharing ONE GPU, against the oracle (the CPU restatement pinned by the
reference's golden vectors).

Like tools/rccl_1gpu_multirank.py, each rank claims its own NCCL_HOSTID so RCCL
accepts P ranks on one device and connects them over its socket transport on
`lo`: this checks the executor's RCCL path (group matching, exact counts,
stream / event hand-offs, chunked pipelines, relay routes) in real processes;
it says nothing about xGMI speed.

For each transport setting (direct; small pipelining chunks; multi-link relay;
relay + flat allgather; flat reduce-scatter + flat allgather; the same on a non-default caller stream with every
collective run twice, the second time into a zeroed output)
it runs all 8 allreduce, 9 reduce_scatter, 2 reduce and 12 allgather
algorithms on fp32 / int64 / int8 at odd sizes, and checks outputs bit for bit
and error statuses against the oracle's return codes.
usage: python tools/rccl_matrix.py [P]   (exit 0 = every rank, every case ok)
"""
import contextlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

CASES = (("float", 4099), ("int64", 1001), ("int8", 333), ("float", 4096),  # 4096: equal blocks up to P = 16
         ("int64", 2048))  # 16-B multiples per block: the one-launch direct form (k_dm_fused) applies
# (name, relay_min_bytes, chunk_bytes, flat phases (1: allgather, 2: reduce-scatter, 4: one-to-all
# exchanges as ncclAllGather, 8: all-peers exchanges as ncclAllToAllv, 16: HIP-graph mode,
# 128: direct peer-memory transport),
# run each collective twice on a side stream)
SETTINGS = (("direct", 0, 0, 0, 0), ("chunk4KiB", 0, 4096, 0, 0), ("relay", 64, 1024, 0, 0),
            ("relay+flat", 64, 1024, 1, 0), ("flatrs+flat", 0, 1024, 3, 0), ("side-stream x2", 64, 1024, 1, 1),
            ("flatrs+flat+collag", 0, 1024, 7, 0), ("flatrs+flat+a2a", 0, 1024, 11, 0),
            ("flat+a2a unchunked", 0, 0, 9, 0),
            # graph mode (bit 16): the first call runs eagerly and is captured, the
            # second (into a zeroed output) is the HIP-graph replay
            ("graphs chunk1KiB x2", 0, 1024, 16, 1), ("graphs relay+flatrs+flat x2", 64, 1024, 16 | 3, 1),
            # the direct peer-memory transport (bit 128) instead of RCCL send/recv
            ("direct-mem", 0, 0, 128, 0), ("direct-mem relay chunk1KiB", 64, 1024, 128, 0),
            ("direct-mem flatrs+flat x2", 0, 1024, 128 | 3, 1),
            # unchunked flat phases over the direct transport: small allreduces
            # whose blocks are 16-B multiples run as ONE k_dm_fused launch
            ("direct-mem flatrs+flat unchunked (fused)", 0, 0, 128 | 3, 0),
            ("direct-mem flatrs+flat unchunked (fused) x2", 0, 0, 128 | 3, 1))


def worker(rank, P, port, q):
    from tools._procs import rank_device
    dev = rank_device(rank)   # (sets the fake RCCL host id on the one-GPU box)
    os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")
    os.environ.setdefault("NCCL_IB_DISABLE", "1")
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(P))
    import numpy as np
    import pico_amd
    import torch
    import torch.distributed as dist
    from oracle import oracle as O
    torch.cuda.set_device(dev)
    dist.init_process_group("gloo")
    comm = pico_amd.Comm.from_torch_distributed(dev)
    npdt = O.NP_DTYPES
    bad, n_ok = [], 0

    def dev(a):
        t = torch.from_numpy(np.ascontiguousarray(a).view(np.uint8).copy()).cuda()
        return t if t.numel() else torch.zeros(16, dtype=torch.uint8, device="cuda")

    def host(t, dt, n):
        return t[: n * np.dtype(npdt[dt]).itemsize].cpu().numpy().view(npdt[dt]).copy()

    def run(tag, want_rc, want, call, out, dt, n):
        nonlocal n_ok
        try:
            call()
            torch.cuda.synchronize()
            comm.synchronize()
            if twice:  # second call into a zeroed output (plan / schedule cache reuse)
                out.zero_()
                call()
                torch.cuda.synchronize()
                comm.synchronize()
            rc = 0
        except pico_amd.BineError:
            rc = 1
        if want_rc != 0:
            if rc == 0:
                bad.append((tag, "expected an error"))
            else:
                n_ok += 1
            return
        if rc != 0:
            bad.append((tag, "error"))
        elif want is not None and not np.array_equal(host(out, dt, n), want):
            bad.append((tag, "data"))
        else:
            n_ok += 1

    side = torch.cuda.Stream()
    for sname, relay, chunk, flat, twice in SETTINGS:
        comm.set_relay(relay)
        comm.set_chunk(chunk)
        comm.set_flat_ag(bool(flat & 1))
        comm.set_flat_rs(bool(flat & 2))
        comm.set_coll_ag(bool(flat & 4))
        comm.set_coll_a2a(bool(flat & 8))
        comm.set_graphs(bool(flat & 16))
        comm.set_direct(bool(flat & 128))
        ctx = torch.cuda.stream(side) if twice else contextlib.nullcontext()
        ctx.__enter__()
        for dt, n in CASES:
            esz = np.dtype(npdt[dt]).itemsize
            sb = O.inputs(dt, n, P)
            for algo in pico_amd.ALGOS["allreduce"]:
                want, rets = O.allreduce(algo, sb, dt, segsize=256)
                r = torch.zeros(n * esz + 16, dtype=torch.uint8, device="cuda")
                s = dev(sb[rank])
                run(f"{sname} allreduce_{algo} {dt} n={n}", rets[rank], want[rank],
                    lambda: pico_amd.allreduce(algo, s, r, n, dt, "sum", comm, segsize=256), r, dt, n)
            rc = [n // P + (i % 3) for i in range(P)]
            sbr = O.inputs(dt, sum(rc), P)
            for algo in pico_amd.ALGOS["reduce_scatter"]:
                want, rets = O.reduce_scatter(algo, sbr, rc, dt)
                r = torch.zeros(rc[rank] * esz + 16, dtype=torch.uint8, device="cuda")
                s = dev(sbr[rank])
                run(f"{sname} reduce_scatter_{algo} {dt} ragged", rets[rank], want[rank],
                    lambda: pico_amd.reduce_scatter(algo, s, r, rc, dt, "sum", comm), r, dt, rc[rank])
            for algo in pico_amd.ALGOS["reduce"]:
                want, rets = O.reduce(algo, sb, dt)
                r = torch.zeros(n * esz + 16, dtype=torch.uint8, device="cuda")
                s = dev(sb[rank])
                run(f"{sname} reduce_{algo} {dt}", rets[rank], want if rank == 0 else None,
                    lambda: pico_amd.reduce(algo, s, r if rank == 0 else None, n, dt, "sum", 0, comm), r, dt, n)
            for algo in pico_amd.ALGOS["allgather"]:
                want, rets = O.allgather(algo, sb, dt)
                r = torch.zeros(P * n * esz + 16, dtype=torch.uint8, device="cuda")
                s = dev(sb[rank])
                run(f"{sname} allgather_{algo} {dt}", rets[rank], want[rank],
                    lambda: pico_amd.allgather(algo, s, r, n, dt, comm), r, dt, P * n)
        ctx.__exit__(None, None, None)
        print(f"rank {rank} {sname}: {n_ok} ok, {len(bad)} bad so far", flush=True)
    comm.set_direct(False)
    # the raw P2P primitive (bine_exchange): ring shift, then all peers at once
    nb = 100003
    mine = torch.full((nb,), rank + 1, dtype=torch.uint8, device="cuda")
    got = torch.zeros(nb, dtype=torch.uint8, device="cuda")
    pico_amd.exchange(comm, [((rank + 1) % P, mine, nb)], [((rank - 1) % P, got, nb)])
    torch.cuda.synchronize()
    ok = bool((got == (rank - 1) % P + 1).all())
    peers = [p for p in range(P) if p != rank]
    allr = torch.zeros(len(peers) * nb, dtype=torch.uint8, device="cuda")
    pico_amd.exchange(comm, [(p, mine, nb) for p in peers], [(p, allr[i * nb:], nb) for i, p in enumerate(peers)])
    torch.cuda.synchronize()
    ok &= all(bool((allr[i * nb:(i + 1) * nb] == p + 1).all()) for i, p in enumerate(peers))
    if ok:
        n_ok += 1
    else:
        bad.append(("exchange", "data"))
    # RCCL's own allreduce (the bench's vendor baseline): int64 SUM is order-free
    vi = [O.fill("int64", nb, 1234 + r) for r in range(P)]
    vs = torch.from_numpy(vi[rank]).to("cuda")
    vr = torch.zeros(nb, dtype=torch.int64, device="cuda")
    pico_amd.vendor_allreduce(vs, vr, nb, "int64", "sum", comm)
    torch.cuda.synchronize()
    want_v = vi[0].copy()
    for x in vi[1:]:
        want_v = want_v + x  # two's complement wrap, as RCCL's int64 add
    if np.array_equal(vr.cpu().numpy(), want_v):
        n_ok += 1
    else:
        bad.append(("vendor_allreduce", "int64"))
    for b in bad[:20]:
        print(f"rank {rank} MISMATCH {b}", flush=True)
    comm.destroy()
    dist.destroy_process_group()
    q.put((rank, n_ok, len(bad)))


if __name__ == "__main__":
    import multiprocessing as mp
    from tools._procs import join_ranks
    P = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=worker, args=(r, P, 29577, q)) for r in range(P)]
    for p in ps:
        p.start()
    join_ranks(ps, 600)
    res = [q.get() for _ in range(sum(1 for p in ps if p.exitcode == 0))]
    print("RESULT P=%d" % P, sorted(res), "exitcodes", [p.exitcode for p in ps], flush=True)
    sys.exit(0 if len(res) == P and all(b == 0 for _, _, b in res) else 1)
