#!/usr/bin/env python3
"""The large-message RCCL path in real processes.

P processes share the one GPU of the test box (distinct NCCL_HOSTIDs: RCCL's
socket transport on `lo`, as tools/rccl_matrix.py) and run
allreduce_bine_bdw_remap on 64 MiB per rank in fp32 and fp64 with the DEFAULT
16 MiB pipelining chunk -- so the chunked two-stream pipeline (receive of chunk
k+1 on the comm stream beside the reduction of chunk k on the compute stream,
the device form of libbine_allreduce.c:1218-1253) runs over real RCCL with
several chunks per step -- for every transport bench.py may pick (direct,
relay, flat, flatrs+flat, +ag, +a2a, trees; and over the direct peer-memory
transport "+dm"), each eagerly and in graph mode
(bine_comm_set_graphs: one eager call + capture, then replays), plus
reduce_scatter_bine_permute_remap
on a 64 MiB input per rank (direct, flatrs, flatrs over the direct transport;
eagerly and in graph mode).  Every rank's output digest is
compared with the committed oracle digests (tests/golden/bench_digests.json,
"L64/..."; trees: the relabelled schedule's); the rank also checks its input's
digest, and a reduce_scatter mismatch reports where the block differs.
usage: python tools/rccl_large.py [P] [DTYPES]   (DTYPES: float,double (default) --
the suite runs fp64 at P = 4 and fp32 at P = 8; exit 0 = every rank, every case ok)
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

N32 = 16_777_216   # 64 MiB fp32
N64 = 8_388_608    # 64 MiB fp64
MODES = ("direct", "relay", "flat", "flatrs+flat", "flatrs+flat+ag", "flatrs+flat+a2a", "trees",
         "direct+dm", "flatrs+flat+dm", "flatrs+flat+dmt", "relay+flat+dm", "trees+dm")
RS_MODES = ("direct", "flatrs", "flatrs+flat+dm", "flatrs+flat+dmt")


ARS = (("float", N32), ("double", N64))


def gkey(coll, algo, dt, n, P, trees=False):
    return f"L64/{coll}/{algo}/{dt}/N{n}/P{P}" + ("/trees" if trees else "")


def expected(P, dts, xdir):
    """the committed oracle digests (tests/golden/bench_digests.json, written by
    tools/make_bench_digests.py in the build container) -- the runtime oracle is
    computed too, checked against them, and its reduce_scatter outputs saved to
    `xdir` so a rank whose output differs can locate the difference"""
    import json
    import numpy as np
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from oracle import oracle as O
    with open(os.path.join(ROOT, "tests", "golden", "bench_digests.json")) as f:
        G = json.load(f)["digests"]
    want = {}
    for dt, n in ARS:
        want[("in", dt)] = G[gkey("input", "fill_pico", dt, n, 8)][:P]
        if dt not in dts:
            continue
        want[("ar", dt, False)] = G[gkey("allreduce", "bine_bdw_remap", dt, n, P)]
        if P in (4, 8):
            want[("ar", dt, True)] = G[gkey("allreduce", "bine_bdw_remap", dt, n, P, True)]
    want[("rs", "float", False)] = G[gkey("reduce_scatter", "bine_permute_remap", "float", N32, P)]
    sb = O.inputs("float", N32, P)
    assert [O.digest(x) for x in sb] == want[("in", "float")], "oracle inputs differ from the committed digests"
    out, rets = O.reduce_scatter("bine_permute_remap", sb, [N32 // P] * P, "float")
    assert not any(rets)
    got = [O.digest(x) for x in out]
    assert got == want[("rs", "float", False)], ("runtime oracle vs committed RS digests", got)
    for r, x in enumerate(out):
        np.save(os.path.join(xdir, f"rs{r}.npy"), x)
    return want


def locate(r, count, path, want_all):
    """where a rank's reduce_scatter output differs from the oracle's: count of
    differing elements, first / last index, NaN count (never written), and
    whether the block equals another rank's expected block (ownership)"""
    import numpy as np
    import pico_amd
    g = r[:count].cpu().numpy()
    e = np.load(path)
    diff = np.flatnonzero(g.view(np.uint32) != e.view(np.uint32))
    d = pico_amd.checksum(r, count, "float")
    owner = [x for x, w in enumerate(want_all) if w == d]
    if diff.size == 0:
        return f"gpu {d:#x}: no element differs"
    i = int(diff[0])
    return (f"gpu {d:#x} expected-owner {owner}: {diff.size} of {count} differ, first {i} (MiB {i * 4 >> 20}) "
            f"gpu {g[i]!r} want {e[i]!r}, last {int(diff[-1])}, NaN {int(np.isnan(g).sum())}")


def worker(rank, P, port, want, dts, q, xdir):
    from tools._procs import rank_device
    dev = rank_device(rank)   # (sets the fake RCCL host id on the one-GPU box)
    os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")
    os.environ.setdefault("NCCL_IB_DISABLE", "1")
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(P))
    import pico_amd
    import torch
    import torch.distributed as dist
    import bench
    torch.cuda.set_device(dev)
    dist.init_process_group("gloo")
    comm = pico_amd.Comm.from_torch_distributed(dev)
    bad, n_ok = [], 0
    side = torch.cuda.Stream()   # graph mode needs a non-NULL caller stream
    modes = [m for m in MODES if (m in bench.transport_modes("auto", P) or m in ("flatrs+flat+a2a", "relay+flat+dm",
                                                                               "trees+dm"))
             and (P in (4, 8) or not m.startswith("trees"))]   # multi-tree: P = 4, 8 only
    for dt, n in ARS:
        if dt not in dts:
            continue
        tdt = {"float": torch.float32, "double": torch.float64}[dt]
        s = torch.empty(n, dtype=tdt, device="cuda")
        r = torch.empty(n, dtype=tdt, device="cuda")
        pico_amd.fill_pico(s, n, dt, 1234 + rank)
        torch.cuda.synchronize()
        din = pico_amd.checksum(s, n, dt)
        if din != want[("in", dt)][rank]:
            bad.append(f"allreduce {dt} INPUT {din:#x} != {want[('in', dt)][rank]:#x} after fill")
        for m in modes:
            for g in (False, True):
                # 0: the library default chunk (16 MiB); graph mode: the first call
                # runs eagerly and is captured (two-stream schedule, the comm stream
                # as the capture's origin), the next ones are replays
                bench.apply_transport(comm, m, 0, g)
                for it in range(3 if g else 2):
                    with torch.cuda.stream(side):
                        r.fill_(float("nan"))
                        pico_amd.allreduce("bine_bdw_remap", s, r, n, dt, "sum", comm)
                    torch.cuda.synchronize()
                    comm.synchronize()
                    d = pico_amd.checksum(r, n, dt)
                    w = want[("ar", dt, m.startswith("trees"))][rank]
                    if d == w:
                        n_ok += 1
                    else:
                        bad.append(f"allreduce {dt} {m} graphs={g} iter {it}: gpu {d:#x} want {w:#x}")
            comm.set_graphs(False)
            print(f"rank {rank} allreduce {dt} {m} (eager + graph): {'ok' if not bad else 'BAD'}", flush=True)
        del s, r
    bench.apply_transport(comm, "direct", 0)
    s = torch.empty(N32, dtype=torch.float32, device="cuda")
    r = torch.empty(N32 // P, dtype=torch.float32, device="cuda")
    pico_amd.fill_pico(s, N32, "float", 1234 + rank)
    torch.cuda.synchronize()
    din = pico_amd.checksum(s, N32, "float")
    if din != want[("in", "float")][rank]:
        bad.append(f"reduce_scatter INPUT {din:#x} != {want[('in', 'float')][rank]:#x} after fill")
    for m in RS_MODES:
        for g in (False, True):
            # graph mode as bench.py's C4 side measurement runs it when the C3
            # trials pick graph replay: one eager call + capture, then replays
            print(f"rank {rank} reduce_scatter {m} graphs={g} ...", flush=True)
            bench.apply_transport(comm, m, 0, g)
            for it in range(3 if g else 1):
                with torch.cuda.stream(side):
                    r.fill_(float("nan"))
                    pico_amd.reduce_scatter("bine_permute_remap", s, r, [N32 // P] * P, "float", "sum", comm)
                torch.cuda.synchronize()
                comm.synchronize()
                if pico_amd.checksum(r, N32 // P, "float") == want[("rs", "float", False)][rank]:
                    n_ok += 1
                else:
                    din = pico_amd.checksum(s, N32, "float")
                    bad.append(f"reduce_scatter {m} graphs={g} iter {it}: "
                               + locate(r, N32 // P, os.path.join(xdir, f"rs{rank}.npy"), want[("rs", "float", False)])
                               + ("" if din == want[("in", "float")][rank] else f"; INPUT now {din:#x}"))
            comm.set_graphs(False)
    for b in bad:
        print(f"rank {rank} MISMATCH {b}", flush=True)
    print(f"rank {rank} rccl {pico_amd.rccl_version()}", flush=True)
    comm.destroy()
    dist.destroy_process_group()
    q.put((rank, n_ok, len(bad)))


if __name__ == "__main__":
    import multiprocessing as mp
    from tools._procs import join_ranks
    P = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    dts = (sys.argv[2] if len(sys.argv) > 2 else "float,double").split(",")
    import tempfile
    xdir = tempfile.mkdtemp(prefix="rccl_large_")
    want = expected(P, dts, xdir)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=worker, args=(r, P, 29591, want, dts, q, xdir)) for r in range(P)]
    for p in ps:
        p.start()
    join_ranks(ps, 600)
    res = [q.get() for _ in range(sum(1 for p in ps if p.exitcode == 0))]
    import shutil
    shutil.rmtree(xdir, ignore_errors=True)
    print("RESULT P=%d" % P, sorted(res), "exitcodes", [p.exitcode for p in ps], flush=True)
    sys.exit(0 if len(res) == P and all(b == 0 for _, _, b in res) else 1)
