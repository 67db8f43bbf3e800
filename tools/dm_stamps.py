#!/usr/bin/env python3
"""Where the direct transport's time goes: C3
(allreduce_bine_bdw_remap fp32 256 MiB per rank) and C4
(reduce_scatter_bine_permute_remap fp32 1 GiB input per rank) over
flatrs+flat+dmt, P processes on the one GPU (distinct NCCL_HOSTIDs), with
per-workgroup wall_clock64 stamps (BINE_DIRECT_STAMPS): for every kind of
workgroup (push, pull, tree) the time spent waiting for the peer's flag and
the time spent copying / reducing, plus the call's timing (bench.timed: max
over ranks, median after dropping 20 %) and its digest check.  Knobs via the
environment (BINE_DIRECT_WGS = push workgroups per message, _PULL_WGS,
_TREE_WGS, BINE_CHUNK_BYTES ...; DM_STAMPS_GRAPHS=1: graph replay); several
settings in one run:
usage: python tools/dm_stamps.py P ITERS SETTING [SETTING ...]
       SETTING = name:VAR=val,VAR=val   (e.g. w128:BINE_DIRECT_WGS=128)
One JSON line per setting.
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

KIND = {0: "push", 1: "pull", 2: "tree", 4: "fused"}   # fused: k_dm_fused, wait = its first phase's wait
TICK_US = 0.01  # wall_clock64: 100 MHz


def summarize(st, calls):
    """per kind: workgroups, wait / work time per workgroup (us, median and
    p90), busy time (union of the workgroups' work intervals) per call"""
    import numpy as np
    if st.shape[0] == 0:
        return {}
    kind = (st[:, 0] >> 24) & 255
    t0 = st[:, 1].astype(np.int64)
    t1 = st[:, 2].astype(np.int64)
    t2 = st[:, 3].astype(np.int64)
    out = {}

    def union(a, b):
        o = np.argsort(a)
        a, b = a[o], b[o]
        tot, cur_a, cur_b = 0, a[0], b[0]
        for x, y in zip(a[1:], b[1:]):
            if x > cur_b:
                tot += cur_b - cur_a
                cur_a, cur_b = x, y
            else:
                cur_b = max(cur_b, y)
        return tot + cur_b - cur_a

    for k, name in KIND.items():
        m = kind == k
        if not m.any():
            continue
        w = (t1[m] - t0[m]) * TICK_US
        c = (t2[m] - t1[m]) * TICK_US
        out[name] = {"wgs_per_call": round(int(m.sum()) / calls, 1),
                     "wait_us_med": round(float(np.median(w)), 2), "wait_us_p90": round(float(np.percentile(w, 90)), 2),
                     "work_us_med": round(float(np.median(c)), 2), "work_us_p90": round(float(np.percentile(c, 90)), 2),
                     "busy_us_per_call": round(union(t1[m], t2[m]) * TICK_US / calls, 1),
                     "span_us_per_call": round(union(t0[m], t2[m]) * TICK_US / calls, 1)}
    # launches: [first workgroup's entry, last workgroup's end]; the gap from
    # one launch's end to the next one's start (launch boundaries, stream
    # waits) and how much of each launch its workgroups spend working
    serial = st[:, 0] >> 32
    spans = {}
    for s_, a_, b_ in zip(serial.tolist(), t0.tolist(), t2.tolist()):
        lo, hi = spans.get(s_, (a_, b_))
        spans[s_] = (min(lo, a_), max(hi, b_))
    seq = sorted(spans.values())
    gaps = [max(0, seq[k + 1][0] - seq[k][1]) * TICK_US for k in range(len(seq) - 1)]
    lens = [(b_ - a_) * TICK_US for a_, b_ in seq]
    out["all"] = {"busy_us_per_call": round(union(t1, t2) * TICK_US / calls, 1),
                  "span_us_per_call": round(union(t0, t2) * TICK_US / calls, 1),
                  "launches_per_call": round(len(spans) / calls, 1),
                  "launch_us_med": round(float(np.median(lens)), 2) if lens else None,
                  "gap_us_med": round(float(np.median(gaps)), 2) if gaps else None,
                  "gap_us_p90": round(float(np.percentile(gaps, 90)), 2) if gaps else None}
    return out


def worker(rank, P, iters, env, port, q):
    os.environ.update(env)
    os.environ.setdefault("BINE_DIRECT_STAMPS", str(1 << 20))
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
    chunk = 0   # the library's default (BINE_CHUNK_BYTES, else 64 MiB over the direct transport)
    res = {}
    for cfg, n, coll in (("C3", bench.C3_ELEMS, "allreduce"), ("C4", bench.C4_ELEMS, "reduce_scatter")):
        sb = torch.empty(n, dtype=torch.float32, device="cuda:0")
        nout = n if coll == "allreduce" else n // P
        rb = torch.empty(nout, dtype=torch.float32, device="cuda:0")
        pico_amd.fill_pico(sb, n, "float", 1234 + rank)
        bench.apply_transport(comm, "flatrs+flat+dmt", chunk, os.environ.get("DM_STAMPS_GRAPHS") == "1")
        rb.fill_(float("nan"))
        if coll == "allreduce":
            fn = lambda: pico_amd.allreduce("bine_bdw_remap", sb, rb, n, "float", "sum", comm, stream=stream)
            key = bench.gkey("C3", "allreduce", "bine_bdw_remap", "float", n, P)
        else:
            fn = lambda: pico_amd.reduce_scatter("bine_permute_remap", sb, rb, [n // P] * P, "float", "sum",
                                                 comm, stream=stream)
            key = bench.gkey("C4", "reduce_scatter", "bine_permute_remap", "float", n, P)
        fn()
        torch.cuda.synchronize()
        comm.direct_stamps(reset=True)
        t = bench.timed(torch, stream, fn, iters, 0, dist, (comm.synchronize,))
        stamps = comm.direct_stamps(reset=True)
        ok, _ = bench.check_digest(pico_amd, rb, nout, "float", key, rank, stream)
        res[cfg] = {"ms": round(t["median_ms"], 4), "host_issue_ms": round(t["issue_ms"], 4),
                    "parity_ok": bench.all_ok(torch, dist, ok), "stamps": summarize(stamps, iters)}
        del sb, rb
        torch.cuda.empty_cache()
    comm.destroy()
    dist.destroy_process_group()
    q.put((rank, res))


def run(P, iters, env, port):
    import multiprocessing as mp
    from tools._procs import join_ranks
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=worker, args=(r, P, iters, env, port, q)) for r in range(P)]
    for p in ps:
        p.start()
    join_ranks(ps, 300)
    res = dict(q.get() for _ in range(sum(1 for p in ps if p.exitcode == 0)))
    return res.get(0), [p.exitcode for p in ps]


if __name__ == "__main__":
    P, iters = int(sys.argv[1]), int(sys.argv[2])
    ok = True
    for i, spec in enumerate(sys.argv[3:]):
        name, _, kv = spec.partition(":")
        env = dict(x.split("=", 1) for x in kv.split(",") if x)
        r0, codes = run(P, iters, env, 29700 + i)
        print(json.dumps({"setting": name, "env": env, "P": P, "rank0": r0, "exitcodes": codes}), flush=True)
        ok = ok and r0 is not None and all(c == 0 for c in codes) and all(
            v["parity_ok"] is not False for v in r0.values())
    sys.exit(0 if ok else 1)
