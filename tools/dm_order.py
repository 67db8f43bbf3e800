#!/usr/bin/env python3
"""Cross-call ordering of the direct peer-memory transport: its
sequence bases live in device memory, so every exchange of one collective
must follow every exchange of the previous one, whichever caller stream
either ran on.  Small collectives (<= 1 MiB) run single-stream on the
caller's stream, large ones on the comm stream: here two processes share the
box's GPU, enable the direct transport, and issue -- with no host
synchronisation in between -- alternating small (C1-sized, 1 MiB fp32) and
large (64 MiB fp32) allreduce_bine_bdw_remap calls on two different caller
streams, then check every output against the oracle's digest.  Without the
cross-stream ordering (bine_comm::order_ev) the small call's k_dm_move and
the large call's first exchange read the same bases and collide.
usage: python tools/dm_order.py [P] [rounds]   (exit 0 = every rank, every call ok)
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

SMALL, LARGE = 262_144, 16_777_216


def expected(P):
    from oracle import oracle as O
    want = {}
    for n in (SMALL, LARGE):
        out, rets = O.allreduce("bine_bdw_remap", O.inputs("float", n, P), "float")
        assert not any(rets)
        want[n] = [O.digest(x) for x in out]
    return want


def worker(rank, P, rounds, port, want, q):
    os.environ["NCCL_HOSTID"] = f"bine-fake-host-{rank}"
    os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")
    os.environ.setdefault("NCCL_IB_DISABLE", "1")
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(P))
    import pico_amd
    import torch
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dist.init_process_group("gloo")
    comm = pico_amd.Comm.from_torch_distributed(0)
    comm.set_direct(True)
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    bufs = {}
    for n in (SMALL, LARGE):
        s = torch.empty(n, dtype=torch.float32, device="cuda:0")
        pico_amd.fill_pico(s, n, "float", 1234 + rank)
        bufs[n] = (s, [torch.empty(n, dtype=torch.float32, device="cuda:0") for _ in range(rounds)])
    torch.cuda.synchronize()
    bad = []
    # call i: size alternates small / large, stream alternates every two
    # calls, so every (size, stream) -> (size, stream) transition occurs
    for i in range(2 * rounds):
        n = SMALL if i % 2 == 0 else LARGE
        st = streams[(i // 2) % 2]
        s, outs = bufs[n]
        with torch.cuda.stream(st):
            outs[i // 2].fill_(float("nan"))
            pico_amd.allreduce("bine_bdw_remap", s, outs[i // 2], n, "float", "sum", comm, stream=st)
    torch.cuda.synchronize()
    comm.synchronize()
    for n in (SMALL, LARGE):
        for k, o in enumerate(bufs[n][1]):
            if pico_amd.checksum(o, n, "float") != want[n][rank]:
                bad.append(f"n={n} call {k}")
    print(f"rank {rank}: {2 * rounds} calls, {len(bad)} mismatches {bad[:4]}", flush=True)
    comm.destroy()
    dist.destroy_process_group()
    q.put((rank, len(bad)))


if __name__ == "__main__":
    import multiprocessing as mp
    from tools._procs import join_ranks
    P = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    want = expected(P)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=worker, args=(r, P, rounds, 29611, want, q)) for r in range(P)]
    for p in ps:
        p.start()
    join_ranks(ps, 240)
    res = [q.get() for _ in range(sum(1 for p in ps if p.exitcode == 0))]
    print("RESULT P=%d" % P, sorted(res), "exitcodes", [p.exitcode for p in ps], flush=True)
    sys.exit(0 if len(res) == P and all(b == 0 for _, b in res) else 1)
