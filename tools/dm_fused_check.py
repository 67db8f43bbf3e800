#!/usr/bin/env python3
"""Whole large collectives as ONE k_dm_fused launch over the direct
peer-memory transport: P processes share the box's GPU,
the transport runs with 1 MiB slots (BINE_DIRECT_SLOT_BYTES) and a 1 MiB
pipelining chunk, so a few MiB per rank already cut the flat reduce-scatter
into several slot-sized chunks -- the multi-chunk program of the kernel
(phase A: every chunk's pushes; B_c: tree c with the allgather's piece c
pushed from registers; D: the allgather's pulls).  Cases: allreduce
bine_bdw_remap / bine_bdw_static / rabenseifner fp32, fp64, int64 SUM / MAX,
exact and ragged chunk counts, in place; reduce_scatter bine_permute_remap
(up to 4 chunks per launch, more in several launches; no allgather); each output bit-exact vs the oracle, and the
number of fused launches counted (bine_comm_fused_calls) -- with the fused
trees off ("+dm") the same calls run the per-exchange launches, and calls of
both forms are interleaved (the two forms move the same messages per pair).
usage: python tools/dm_fused_check.py [P]   (exit 0 = every rank, every case ok)
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

SLOT = 1 << 20


def cases(P):
    """(coll, algo, dtype, op, count per rank (allreduce) or block (RS), in place, fused expected)"""
    per = SLOT // 4   # fp32 elements per slot
    out = []
    for dt, esz in (("float", 4), ("double", 8), ("int64", 8)):
        e = SLOT // esz
        out.append(("allreduce", "bine_bdw_remap", dt, "sum", 2 * P * e, False, True))     # 2 full chunks
        out.append(("allreduce", "bine_bdw_remap", dt, "sum", P * e + P * 64, False, True))  # 1 full + a short one
    out.append(("allreduce", "bine_bdw_remap", "int64", "max", P * (SLOT // 8), False, True))
    out.append(("allreduce", "bine_bdw_remap", "float", "sum", 2 * P * per, True, True))      # in place
    out.append(("allreduce", "bine_bdw_static", "float", "sum", 2 * P * per, False, True))
    out.append(("allreduce", "rabenseifner", "double", "sum", P * (SLOT // 8) + 8 * P, False, True))
    out.append(("allreduce", "bine_bdw_remap", "float", "sum", 3 * P * per, False, False))    # 3 chunks + AG: > 4 slots
    out.append(("reduce_scatter", "bine_permute_remap", "float", "sum", 4 * per, False, True))  # 4 chunks, no AG
    out.append(("reduce_scatter", "bine_permute_remap", "double", "sum", 3 * (SLOT // 8) - 2, False, True))
    # more chunks than one launch holds: one launch per 4 chunks
    out.append(("reduce_scatter", "bine_permute_remap", "float", "sum", 6 * per, False, True))
    out.append(("reduce_scatter", "bine_permute_remap", "int64", "sum", 9 * (SLOT // 8) + 2, False, True))
    return out


def worker(rank, P, port, q):
    from tools._procs import rank_device
    dev = rank_device(rank)   # (sets the fake RCCL host id on the one-GPU box)
    os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")
    os.environ.setdefault("NCCL_IB_DISABLE", "1")
    os.environ["BINE_DIRECT_SLOT_BYTES"] = str(SLOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(P))
    import numpy as np
    import pico_amd
    import torch
    import torch.distributed as dist
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from oracle import oracle as O
    torch.cuda.set_device(dev)
    dist.init_process_group("gloo")
    comm = pico_amd.Comm.from_torch_distributed(dev)
    comm.set_direct(True)
    comm.set_flat_ag(True)
    comm.set_flat_rs(True)
    comm.set_chunk(SLOT)
    side = torch.cuda.Stream()
    bad, n_ok = [], 0
    for tree in (1, 0, 1):   # fused trees on: one launch; off: per-exchange launches; on again
        comm.set_direct_tree(tree)
        for coll, algo, dt, op, n, inplace, fused in cases(P):
            np_dt = O.NP_DTYPES[dt]
            esz = np.dtype(np_dt).itemsize
            if coll == "allreduce":
                sb = O.inputs(dt, n, P)
                want, rets = O.allreduce(algo, sb, dt, op)
                want = want[rank]
                total, outn = n, n
            else:
                sb = O.inputs(dt, n * P, P)
                want, rets = O.reduce_scatter(algo, sb, [n] * P, dt, op)
                want = want[rank]
                total, outn = n * P, n
            assert not any(rets)
            s = torch.from_numpy(sb[rank].view(np.uint8).copy()).to("cuda")
            r = torch.full((outn * esz,), 0xA5, dtype=torch.uint8, device="cuda")
            if inplace:
                r = s.clone()
            torch.cuda.synchronize()
            before = comm.fused_calls()
            with torch.cuda.stream(side):
                src = pico_amd.IN_PLACE if inplace else s
                if coll == "allreduce":
                    pico_amd.allreduce(algo, src, r, n, dt, op, comm)
                else:
                    pico_amd.reduce_scatter(algo, src, r, [n] * P, dt, op, comm)
            torch.cuda.synchronize()
            comm.synchronize()
            got = r[:outn * esz].cpu().numpy().view(np_dt)
            took = comm.fused_calls() - before
            tag = f"{coll} {algo} {dt} {op} n={n} inplace={inplace} trees={tree}"
            ok = got.tobytes() == np.ascontiguousarray(want).tobytes()
            if ok and took != (1 if fused and tree else 0):
                ok = False
                tag += f" (fused launches {took}, expected {1 if fused and tree else 0})"
            if ok:
                n_ok += 1
            else:
                diff = np.flatnonzero(got.view(np.uint8) != np.ascontiguousarray(want).view(np.uint8))
                bad.append(f"{tag}: {diff.size} bytes differ, first {diff[:1]}")
    for b in bad:
        print(f"rank {rank} MISMATCH {b}", flush=True)
    print(f"rank {rank}: {n_ok} ok, {len(bad)} bad", flush=True)
    comm.destroy()
    dist.destroy_process_group()
    q.put((rank, n_ok, len(bad)))


if __name__ == "__main__":
    import multiprocessing as mp
    from tools._procs import join_ranks
    P = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=worker, args=(r, P, 29631, q)) for r in range(P)]
    for p in ps:
        p.start()
    join_ranks(ps, 240)
    res = [q.get() for _ in range(sum(1 for p in ps if p.exitcode == 0))]
    print("RESULT P=%d" % P, sorted(res), "exitcodes", [p.exitcode for p in ps], flush=True)
    sys.exit(0 if len(res) == P and all(b == 0 for _, _, b in res) else 1)
