#!/usr/bin/env python3
"""Benchmark of the MI355X Bine reduce-family path (BASELINE.json metric:
"device-resident fp32 allreduce GB/s per rank @256 MiB, 1/2/4/8 MI355X").

Every N measures the metric's own workload, BASELINE config C3:
allreduce_bine_bdw_remap, fp32 SUM, 256 MiB (67,108,864 elements) per rank,
inputs resident in HBM (pico_core's rand_r distribution, seed 1234 + rank,
generated on the device), `value` = per-rank algorithmic bandwidth S / t.

* N = 1: a size-1 RCCL communicator.  The reference's P = 1 allreduce is its
  sbuf -> rbuf copy (libbine_allreduce.c:849-852), here one k_copy launch;
  roofline = HBM, 2 S bytes per launch.  The C2 reduce kernel, the flat
  reduce-scatter's tree kernel and the reduce kernel at small windows are
  reported as side kernels, each with its own roofline and parity check.
* N > 1 (torch.distributed.run, one process per GPU): RCCL P2P over xGMI.
  Every transport (the literal schedule and its bit-identical multi-link
  forms) is timed briefly and CHECKED (digest of every rank's output against
  tests/golden/bench_digests.json, the oracle's values for these exact inputs);
  a transport whose output is wrong is excluded.  The fastest correct
  transport x pipelining chunk is then timed and checked again, and C1, C4, C5
  run on it, each checked the same way.

Statistic (the reference's: pico_core/pico_core.c:133-140,
plot/summarize_data.py:24-48): an event pair per iteration on the stream the
collective is issued on (K iterations back to back between a barrier +
device synchronize on both sides), the max over ranks per iteration, the
first 20 % dropped, the median.  One JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import json
import re
import os
import platform
import statistics
import sys
import threading
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md, chip-level parameters (spec)
XGMI_LINK_GBS = 153.0          # one xGMI link (task statement); 7 links per GPU
TARGET_BUSBW_GBS = 7 * XGMI_LINK_GBS   # BASELINE.json north_star: min(HBM, per-rank xGMI) = 1071 GB/s
METRIC = "device-resident fp32 allreduce GB/s per rank @256 MiB, 1/2/4/8 MI355X"
C1_ELEMS = 262_144             # 1 MiB fp32
C2_ELEMS = 16_777_216          # 64 MiB fp32
C3_ELEMS = 67_108_864          # 256 MiB fp32
C4_ELEMS = 268_435_456         # 1 GiB fp32 reduce_scatter input per rank
C5_ELEMS = 33_554_432          # 256 MiB of fp64 / int64
TREE_LEAVES, TREE_ELEMS, TREE_SEED = 8, 4_194_304, 5000   # flat reduce-scatter at C3, P = 8, 16 MiB chunks
MIB = 1 << 20
WARMUP_DROP = 0.2              # plot/summarize_data.py:24 warmup_ratio
GOLDEN = os.path.join(ROOT, "tests", "golden", "bench_digests.json")
REF_BENCH = os.path.join(ROOT, "oracle", "_ref", "ref_bench")
MPIEXEC = "/opt/conda/bin/mpiexec"


# ---- host / runtime facts ---------------------------------------------------------

def host_info():
    model = platform.processor() or ""
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else None
    return {"cpu_model": model, "nproc": os.cpu_count(), "cpus_usable": aff}


def kernels_source_sha256():
    import hashlib
    with open(os.path.join(ROOT, "pico_amd", "csrc", "kernels.hip"), "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()


def _pmc_traffic(kernel_prefix: str):
    """HBM bytes per launch of a kernel from the committed rocprofv3 PMC passes
    (profiles/latest_pmc.json, written by tools/pmc_summary.py), or None -- also
    when those passes were taken on another build: the file carries the sha256
    of the kernels.hip it measured, and a tree whose kernels.hip differs gets
    None rather than a stale figure."""
    try:
        with open(os.path.join(ROOT, "profiles", "latest_pmc.json")) as f:
            pmc = json.load(f)
        if pmc.get("kernels_hip_sha256") != kernels_source_sha256():
            return None
        return float(pmc["kernels"][kernel_prefix]["hbm_bytes_per_launch"])
    except Exception:
        return None


# ---- parity: committed oracle digests --------------------------------------------

_GOLD = None


def golden(key: str):
    """per-rank digests for `key` (tools/make_bench_digests.py), or None"""
    global _GOLD
    if _GOLD is None:
        try:
            with open(GOLDEN) as f:
                _GOLD = json.load(f)["digests"]
        except OSError:
            _GOLD = {}
    return _GOLD.get(key)


def gkey(cfg, coll, algo, dtype, n, P, trees=False):
    return f"{cfg}/{coll}/{algo}/{dtype}/N{n}/P{P}" + ("/trees" if trees else "")


def check_digest(pico_amd, buf, count, dtype, key, rank, stream=None):
    """(ok, digest): bine_checksum of the device buffer vs the committed oracle
    digest of this rank (ok None when no golden entry exists)"""
    d = pico_amd.checksum(buf, count, dtype, stream=stream)
    want = golden(key)
    return (None if want is None else d == int(want[rank])), d


def all_ok(torch, dist, ok):
    """every rank's verdict (None = unchecked counts as not failed)"""
    if dist is None:
        return ok
    t = torch.tensor([0 if ok is False else 1, 1 if ok is None else 0], dtype=torch.int64)
    dist.all_reduce(t, op=dist.ReduceOp.MIN)
    if int(t[0]) == 0:
        return False
    return None if int(t[1]) == 1 and ok is None else True


# ---- timing (the reference's statistic) --------------------------------------------

def timed(torch, stream, call, steps, warmup, dist=None, syncs=(), per_iter=True):
    """K iterations of call() back to back between a barrier + device
    synchronize on both sides.  per_iter: each iteration bracketed by its own
    event pair on `stream`; per iteration the max over ranks; the first 20 %
    dropped; the median (pico_core.c:133-140, summarize_data.py:24-48).
    Always: one event pair around the whole timed region, region_ms = its
    time / K (the average launch duration a kernel-trace profile reports for
    single-kernel calls; per-iteration events add a dispatch bubble each).
    Returns {median_ms, mean_ms (of the kept samples), min_ms, max_ms, samples,
    region_ms, issue_ms (host time per call spent enqueueing, max over ranks),
    wall_s}; without per_iter the per-iteration fields are region_ms."""
    def sync():
        torch.cuda.synchronize()
        for s in syncs:
            s()
    for _ in range(warmup):
        call()
    sync()
    if dist is not None:
        dist.barrier()
    sync()
    ev = lambda: torch.cuda.Event(enable_timing=True)  # noqa: E731
    evs = [(ev(), ev()) for _ in range(steps)] if per_iter else []
    r0, r1 = ev(), ev()
    issue = 0.0
    t0 = time.perf_counter()
    r0.record(stream)
    for i in range(steps):
        if per_iter:
            evs[i][0].record(stream)
        ti = time.perf_counter()
        call()
        issue += time.perf_counter() - ti
        if per_iter:
            evs[i][1].record(stream)
    r1.record(stream)
    sync()
    wall = time.perf_counter() - t0
    if dist is not None:
        dist.barrier()
    return reduce_stats(torch, dist, [a.elapsed_time(b) for a, b in evs], r0.elapsed_time(r1) / steps,
                        issue * 1e3 / steps, wall)


class Drain:
    """comm.synchronize as a timed() sync that never raises: since round 6 the
    completion of calls whose direct-transport wait timed out is an error on
    the rank that timed out (bine_comm_synchronize) -- and
    possibly only there.  Raising on that rank alone would leave the ranks in
    different collectives (timed()'s barriers, the digest votes), so the first
    error is recorded here and `failed()` agrees on it over all ranks."""

    def __init__(self, comm):
        self.comm = comm
        self.err = None

    def __call__(self):
        import pico_amd
        try:
            self.comm.synchronize()
        except pico_amd.BineError as e:
            if self.err is None:
                self.err = str(e)

    def guard(self, call):
        """call() with its issue-time library error recorded, not raised (a
        poisoned transport refuses a call at issue on the rank that timed out
        while its peers issue theirs); nothing more is issued on this rank
        once it failed"""
        import pico_amd

        def g():
            if self.err is not None:
                return
            try:
                call()
            except pico_amd.BineError as e:
                self.err = str(e)
        return g

    def failed(self, dist):
        """None when no rank saw an error, else every such rank's error --
        'rank r: <its error>' joined by ' || ', lowest rank first; a
        direct-transport timeout carries the waiter's record and both ends'
        flags and bases (DirectState::describe), so the line says which wait
        of which rank stalled on what -- plus the box's queue census
        (VERDICT r5 item 3).  Collective: every rank gets the same answer."""
        if dist is None:
            errs = [self.err]
        else:
            errs = [None] * dist.get_world_size()
            dist.all_gather_object(errs, self.err)
        bad = [f"rank {r}: {e[:1500]}" for r, e in enumerate(errs) if e is not None]
        if not bad:
            return None
        return " || ".join(bad) + " || " + queue_census()


def queue_census():
    """compute queues per process on the box's GPUs (KFD sysfs), in one line:
    how many user-mode queues the scheduler has to place when a wait times
    out (past the hardware's slots it time-slices them)"""
    try:
        base = "/sys/class/kfd/kfd/proc"
        per = {}   # gpu_id -> [compute queues of each process on it]
        for pid in sorted(os.listdir(base)):
            qd = os.path.join(base, pid, "queues")
            if not os.path.isdir(qd):
                continue
            mine = {}
            for q in os.listdir(qd):
                with open(os.path.join(qd, q, "type")) as f:
                    if f.read().strip() != "0":
                        continue
                with open(os.path.join(qd, q, "gpuid")) as f:
                    g = f.read().strip()
                mine[g] = mine.get(g, 0) + 1
            for g, n in mine.items():
                per.setdefault(g, []).append(n)
        hqd = hw_queue_slots()
        # KFD's sysfs is the host's: other jobs on the host's other GPUs show too
        return ("KFD compute queues per GPU (gpu_id: total in processes [per process], HW queue slots): "
                + "; ".join(f"{g}: {sum(v)} in {len(v)} {v}, slots {hqd.get(g, '?')}" for g, v in sorted(per.items())))
    except OSError as e:
        return f"KFD compute queues: unreadable ({e})"


def hw_queue_slots():
    """gpu_id -> the compute queue slots KFD reports for that GPU
    (topology `num_cp_queues`): past that many user queues on one GPU the
    scheduler time-slices them"""
    out = {}
    base = "/sys/class/kfd/kfd/topology/nodes"
    try:
        for node in os.listdir(base):
            try:
                with open(os.path.join(base, node, "gpu_id")) as f:
                    g = f.read().strip()
                with open(os.path.join(base, node, "properties")) as f:
                    props = dict(line.split()[:2] for line in f if len(line.split()) >= 2)
            except OSError:
                continue
            if g != "0" and "num_cp_queues" in props:
                out[g] = int(props["num_cp_queues"])
    except OSError:
        pass
    return out


def measure(torch, stream, dist, comm, call, steps, warmup):
    """timed() of a collective with every rank's library errors agreed on:
    (stats, None) or (stats, 'rank r: <error>') -- the same on every rank"""
    d = Drain(comm)
    st = timed(torch, stream, d.guard(call), steps, warmup, dist, (d,))
    return st, d.failed(dist)


def reduce_stats(torch, dist, per, region, issue_ms, wall):
    """the statistic over ranks: per iteration the max over ranks (as every
    other figure), the first 20 % of iterations dropped, the median of the
    rest (pico_core.c:133-140, summarize_data.py:24-48); `per` empty = no
    per-iteration events (the region average stands for every field)"""
    t = torch.tensor(list(per) + [region, issue_ms, wall], dtype=torch.float64)
    if dist is not None:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    n = len(per)
    region = float(t[n])
    vals = [float(x) for x in t[:n]] or [region]
    kept = vals[int(len(vals) * WARMUP_DROP):] or vals
    return {"median_ms": statistics.median(kept), "mean_ms": statistics.fmean(kept), "min_ms": min(kept),
            "max_ms": max(kept), "samples": len(kept) if n else 0, "region_ms": region,
            "issue_ms": float(t[n + 1]), "wall_s": float(t[n + 2])}


class quiet_stdout:
    """fd 1 -> fd 2 while RCCL initialises a communicator: RCCL prints its
    version banner on stdout, and bench.py's stdout is one JSON line"""
    def __enter__(self):
        sys.stdout.flush()
        self.saved = os.dup(1)
        os.dup2(2, 1)
        return self

    def __exit__(self, *exc):
        sys.stdout.flush()
        os.dup2(self.saved, 1)
        os.close(self.saved)
        return False


def _r(x, n=4):
    return None if x is None else round(x, n)


# ---- CPU baseline (rank 0, N = 1) --------------------------------------------------

def _ref_bench(np_: int, args, timeout: float):
    """oracle/_ref/ref_bench (the real reference libbine + MPICH, built from the
    reference sources by `make -C oracle ref`) under mpiexec as a child
    process; its JSON line, or None."""
    import subprocess
    env = dict(os.environ)
    env["PATH"] = "/opt/conda/bin:" + env.get("PATH", "")
    r = subprocess.run([MPIEXEC, "-n", str(np_), REF_BENCH] + [str(a) for a in args], env=env,
                       capture_output=True, text=True, timeout=timeout)
    if r.returncode != 0:
        return None
    for line in r.stdout.splitlines():
        if line.startswith("{"):
            return json.loads(line)
    return None


def cpu_baseline(gpu_digest=None, budget_s: float = 5.0):
    """The same workload on the box's host cores: the REAL reference libbine's
    allreduce_bine_bdw_remap (oracle/_ref/ref_bench, compiled from the
    reference sources against MPICH 3.3.2) on 256 MiB fp32 per rank at P = 1
    (`value`: the single-GPU line's comparison), and at P = 2, 4, 8 host ranks
    (one per core), same statistic; its output digest is compared with the
    GPU's and the oracle's.  Plus C1 (the reference's own CPU configuration),
    C4 (reduce_scatter_bine_permute_remap, 1 GiB fp32 per rank) and C5
    (allreduce_bine_bdw_remap fp64 / int64, 256 MiB per rank) at P = 8 host
    ranks, each digest-checked, and MPICH's MPI_Reduce_local on C2 (libbine's
    arithmetic).  Falls back to the oracle's restatement (kind "port") when
    the reference build is absent."""
    S = C3_ELEMS * 4
    host = host_info()
    if not (os.path.exists(REF_BENCH) and os.path.exists(MPIEXEC)):
        return cpu_baseline_port(budget_s, host)
    c3 = {}
    for p in (1, 2, 4, 8):
        try:
            ar = _ref_bench(p, ["allreduce", "bine_bdw_remap", C3_ELEMS, 10 if p == 1 else 5], 180)
        except Exception:
            ar = None
        if ar and ar.get("rc") == 0:
            t = ar["median_s"]
            want = golden(gkey("C3", "allreduce", "bine_bdw_remap", "float", C3_ELEMS, p))
            c3[f"P{p}"] = {"ms": round(t * 1e3, 3), "algbw_per_rank_GBs": round(S / t / 1e9, 3),
                           "busbw_per_rank_GBs": round(2 * (p - 1) / p * S / t / 1e9, 3), "cores": p,
                           "iterations": ar["iters"],
                           "output_digest_equals_oracle": (None if want is None
                                                           else int(ar["digest"]) == int(want[0]))}
            if p == 1 and gpu_digest is not None:
                c3["P1"]["output_digest_equals_gpu"] = int(ar["digest"]) == int(gpu_digest)
    if "P1" not in c3:
        return cpu_baseline_port(budget_s, host)
    out = {"value": c3["P1"]["algbw_per_rank_GBs"], "unit": "GB/s", "cores": 1, "kind": "reference",
           "sample": (f"real libbine allreduce_bine_bdw_remap fp32 256 MiB, P = 1 host rank (its sbuf->rbuf "
                      f"copy, libbine_allreduce.c:849-852), {c3['P1']['iterations']} iterations, median after "
                      f"dropping the first 20 %: {c3['P1']['ms']} ms"),
           "host": dict(host, mpi="MPICH 3.3.2 (/opt/conda), mpiexec Hydra, one rank per core"),
           "libbine_allreduce_bine_bdw_remap_c3": c3}
    try:
        c1 = _ref_bench(4, ["allreduce", "bine_bdw_remap", C1_ELEMS, 200], 120)
    except Exception:
        c1 = None
    if c1 and c1.get("rc") == 0:
        out["libbine_allreduce_bine_bdw_remap_c1_P4"] = {"us": round(c1["median_s"] * 1e6, 2), "cores": 4,
                                                          "iterations": 200}
    # BASELINE configs C4 and C5 on the host cores: the
    # reference's reduce_scatter_bine_permute_remap on 1 GiB fp32 per rank and
    # its allreduce_bine_bdw_remap on 256 MiB of fp64 / int64 per rank, both
    # at P = 8 host ranks (one per core), the same statistic, rank 0's output
    # digest against the committed oracle digest
    for name, args, key, S_ in (
            ("libbine_reduce_scatter_bine_permute_remap_c4_P8",
             ["reduce_scatter", "bine_permute_remap", C4_ELEMS, 3],
             gkey("C4", "reduce_scatter", "bine_permute_remap", "float", C4_ELEMS, 8), C4_ELEMS * 4),
            ("libbine_allreduce_bine_bdw_remap_c5_double_P8",
             ["allreduce", "bine_bdw_remap", C5_ELEMS, 5, "double"],
             gkey("C5", "allreduce", "bine_bdw_remap", "double", C5_ELEMS, 8), C5_ELEMS * 8),
            ("libbine_allreduce_bine_bdw_remap_c5_int64_P8",
             ["allreduce", "bine_bdw_remap", C5_ELEMS, 5, "int64"],
             gkey("C5", "allreduce", "bine_bdw_remap", "int64", C5_ELEMS, 8), C5_ELEMS * 8)):
        try:
            r = _ref_bench(8, args, 180)
        except Exception:
            r = None
        if r and r.get("rc") == 0:
            t = r["median_s"]
            want = golden(key)
            rs = args[0] == "reduce_scatter"
            out[name] = {"ms": round(t * 1e3, 3), "cores": 8, "iterations": r["iters"],
                         ("busbw_per_rank_GBs" if rs else "algbw_per_rank_GBs"):
                             round((7 / 8 if rs else 1.0) * S_ / t / 1e9, 3),
                         "output_digest_equals_oracle": None if want is None else int(r["digest"]) == int(want[0])}
        else:
            out[name] = {"error": "ref_bench failed" if r is None else f"rc {r.get('rc')}"}
    try:
        rl = _ref_bench(1, ["reduce_local", C2_ELEMS, budget_s], budget_s + 60)
    except Exception:
        rl = None
    if rl:
        per = rl["s_per_call"]
        out["mpich_reduce_local_c2"] = {"GBs": round(3 * C2_ELEMS * 4 / per / 1e9, 3), "ms_per_call": round(per * 1e3, 3),
                                        "calls": rl["calls"], "cores": 1}
    return out


def cpu_baseline_port(budget_s: float, host):
    """the oracle's allreduce_bine_bdw_remap at P = 1 on the C3 buffer (its copy)"""
    import numpy as np
    from oracle import oracle as O
    sb = [O.fill("float", C3_ELEMS, 1234)]
    n, t0, ts = 0, time.perf_counter(), []
    while time.perf_counter() - t0 < budget_s and n < 50:
        t1 = time.perf_counter()
        O.allreduce("bine_bdw_remap", sb, "float")
        ts.append(time.perf_counter() - t1)
        n += 1
    t = float(np.median(ts[int(len(ts) * WARMUP_DROP):] or ts))
    return {"value": round(C3_ELEMS * 4 / t / 1e9, 3), "unit": "GB/s", "cores": 1, "kind": "port",
            "sample": f"oracle allreduce_bine_bdw_remap fp32 256 MiB P = 1, {n} calls, median {t * 1e3:.2f} ms",
            "host": host}


# ---- N = 1 ------------------------------------------------------------------------

def _side_reduce(torch, pico_amd, dev, stream, steps, warmup):
    """C2: the MPI_Reduce_local kernel, inout = inout + in on 64 MiB fp32, 4
    rotating buffer sets (768 MiB, beyond the 256 MiB Infinity Cache); then
    one call on fresh inputs (seeds 1234 / 1235) checked against the oracle."""
    sets = 4
    ins, ios = [], []
    for k in range(sets):
        a = torch.empty(C2_ELEMS, dtype=torch.float32, device=dev)
        b = torch.empty(C2_ELEMS, dtype=torch.float32, device=dev)
        pico_amd.fill_pico(a, C2_ELEMS, "float", 1234 + 2 * k)
        pico_amd.fill_pico(b, C2_ELEMS, "float", 1235 + 2 * k)
        ins.append(a)
        ios.append(b)
    i = [0]

    def call():
        pico_amd.reduce_local(ins[i[0] % sets], ios[i[0] % sets], C2_ELEMS, "float", "sum", stream=stream)
        i[0] += 1
    st = timed(torch, stream, call, steps, warmup, per_iter=False)
    pico_amd.fill_pico(ins[0], C2_ELEMS, "float", 1234)
    pico_amd.fill_pico(ios[0], C2_ELEMS, "float", 1235)
    pico_amd.reduce_local(ins[0], ios[0], C2_ELEMS, "float", "sum", stream=stream)
    ok, _ = check_digest(pico_amd, ios[0], C2_ELEMS, "float", f"C2/reduce_local/sum/float/N{C2_ELEMS}", 0)
    del ins, ios
    torch.cuda.empty_cache()
    alg = 3 * C2_ELEMS * 4
    return {"kernel": "bine::k_reduce<float,SUM>", "workload": "C2: fp32 inout += in, 64 MiB, 1 GPU",
            "parity_ok": ok, "us_per_launch": round(st["region_ms"] * 1e3, 3), "launches": steps,
            "roofline": {"bound": "hbm", "achieved": round(alg / (st["region_ms"] * 1e-3) / 1e9, 1),
                         "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(alg / (st["region_ms"] * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                         "traffic": _pmc_traffic("k_reduce"), "algorithmic_bytes_per_launch": alg}}


def _side_tree(torch, pico_amd, dev, stream, steps, warmup):
    """the flat reduce-scatter's tree kernel at its C3 shape (8 leaves x 16 MiB
    -> 16 MiB; 9 x 16 MiB per launch), 4 rotating sets; set 0 = leaf j seeded
    5000 + j, checked against the oracle's pairwise tree"""
    sets = 4
    bufs = []
    for k in range(sets):
        leaves = [torch.empty(TREE_ELEMS, dtype=torch.float32, device=dev) for _ in range(TREE_LEAVES)]
        for j, t in enumerate(leaves):
            pico_amd.fill_pico(t, TREE_ELEMS, "float", TREE_SEED + 16 * k + j)
        bufs.append((leaves, torch.empty(TREE_ELEMS, dtype=torch.float32, device=dev)))
    i = [0]

    def call():
        leaves, out = bufs[i[0] % sets]
        rc = pico_amd.reduce_tree(leaves, out, TREE_ELEMS, "float", "sum", stream=stream)
        assert rc == 0, rc
        i[0] += 1
    st = timed(torch, stream, call, steps, warmup, per_iter=False)
    ok, _ = check_digest(pico_amd, bufs[0][1], TREE_ELEMS, "float",
                         f"tree/reduce_tree/sum/float/N{TREE_ELEMS}/L{TREE_LEAVES}", 0)
    del bufs
    torch.cuda.empty_cache()
    alg = (TREE_LEAVES + 1) * TREE_ELEMS * 4
    return {"kernel": "bine::k_reduce_tree<float,SUM,8>", "leaves": TREE_LEAVES, "elems_per_leaf": TREE_ELEMS,
            "parity_ok": ok, "us_per_launch": round(st["region_ms"] * 1e3, 3), "launches": steps,
            "roofline": {"bound": "hbm", "achieved": round(alg / (st["region_ms"] * 1e-3) / 1e9, 1),
                         "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(alg / (st["region_ms"] * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                         "traffic": _pmc_traffic("k_reduce_tree"), "algorithmic_bytes_per_launch": alg}}


def _side_small_windows(torch, pico_amd, dev, stream):
    """k_reduce at the windows of C1 and of pipelines' tail chunks: 64
    launches over 16 rotating windows of a 1 GiB region, captured once into a
    HIP graph and replayed, so the launches run back to back with the host out
    of the loop (the executor issues them from C++; issued one by one from
    Python through ctypes they would measure the interpreter).  Per window:
    time per launch incl. the launch-to-launch boundary, HBM GB/s, fraction."""
    region = 1 << 28   # elements (1 GiB fp32) per operand
    a = torch.empty(region, dtype=torch.float32, device=dev)
    b = torch.empty(region, dtype=torch.float32, device=dev)
    pico_amd.fill_pico(a, region, "float", 7)
    pico_amd.fill_pico(b, region, "float", 8)
    torch.cuda.synchronize()
    out = {}
    launches = 64
    for w in (256 << 10, 1 << 20, 4 << 20, 16 << 20):
        n = w // 4
        g = torch.cuda.CUDAGraph()
        cs = torch.cuda.Stream(dev)
        with torch.cuda.graph(g, stream=cs):
            for i in range(launches):
                off = (i % 16) * (region // 16)
                pico_amd.reduce_local(a[off:], b[off:], n, "float", "sum", stream=cs)
        st = timed(torch, stream, g.replay, 8, 2, per_iter=False)
        us = st["region_ms"] * 1e3 / launches
        gbs = 3 * w / (us * 1e-6) / 1e9
        out[f"{w >> 10}KiB"] = {"us_per_launch": round(us, 3), "GBs": round(gbs, 1), "frac": round(gbs / HBM_PEAK_GBS, 4)}
        del g
    del a, b
    torch.cuda.empty_cache()
    return out


def bench_n1(steps: int, warmup: int, want_cpu: bool, cpu_budget: float):
    import pico_amd
    import torch
    dev = torch.device("cuda:0")
    torch.cuda.set_device(0)
    with quiet_stdout():
        comm = pico_amd.Comm.rccl(0, 1, pico_amd.Comm.unique_id(), 0)
    n = C3_ELEMS
    S = n * 4
    sbuf = torch.empty(n, dtype=torch.float32, device=dev)
    rbuf = torch.zeros(n, dtype=torch.float32, device=dev)
    pico_amd.fill_pico(sbuf, n, "float", 1234)
    torch.cuda.synchronize()
    stream = torch.cuda.current_stream(dev)
    call = lambda: pico_amd.allreduce("bine_bdw_remap", sbuf, rbuf, n, "float", "sum", comm,  # noqa: E731
                                      stream=stream)
    st = timed(torch, stream, call, steps, warmup, syncs=(comm.synchronize,))
    # the kernel's average launch duration for the roofline: the same K calls
    # back to back with one event pair around them (per-iteration events add a
    # dispatch bubble each; this is what a kernel-trace average reports)
    st_k = timed(torch, stream, call, steps, 2, syncs=(comm.synchronize,), per_iter=False)
    key = gkey("C3", "allreduce", "bine_bdw_remap", "float", n, 1)
    ok, dig = check_digest(pico_amd, rbuf, n, "float", key, 0)
    ok_in, _ = check_digest(pico_amd, sbuf, n, "float", key, 0)   # input untouched (P = 1: output == input)
    comm.destroy()
    del sbuf, rbuf
    torch.cuda.empty_cache()
    ms = st["median_ms"]
    algbw = S / (ms * 1e-3) / 1e9
    hbm = 2 * S / (st_k["region_ms"] * 1e-3) / 1e9
    side = {"k_reduce_C2": _side_reduce(torch, pico_amd, dev, stream, steps, warmup),
            "k_reduce_tree_C3_flat_rs_chunk": _side_tree(torch, pico_amd, dev, stream, steps, warmup)}
    if os.environ.get("BENCH_NO_SMALL_WINDOWS") != "1":   # PMC passes: one k_reduce shape only
        side["k_reduce_small_windows"] = _side_small_windows(torch, pico_amd, dev, stream)
    out = {
        "metric": METRIC, "value": round(algbw, 2), "unit": "GB/s", "n_gpus": 1, "steps": steps, "warmup": warmup,
        "ms_per_step": round(ms, 5), "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "dtype": "f32", "data": "synthetic (pico_core rand_r distribution, seed 1234 + rank, generated on device)",
        "config": {"workload": "C3 at P = 1: allreduce_bine_bdw_remap fp32 SUM 256 MiB/rank (67,108,864 elem) "
                               "through a size-1 RCCL communicator = the reference's sbuf->rbuf copy "
                               "(libbine_allreduce.c:849-852), device-resident, 1 MI355X",
                   "value_definition": "per-rank algbw = S / t, t = median after dropping the first 20 % of "
                                       "per-iteration event times (pico_core.c:133-140, summarize_data.py:24-48)",
                   "stats_ms": {k: _r(v, 5) for k, v in st.items()},
                   "parity": {"ok": bool(ok) and bool(ok_in), "check": "bine_checksum(rbuf) == oracle digest "
                              f"{key} (tests/golden/bench_digests.json), input untouched", "digest": str(dig)},
                   "rccl": pico_amd.rccl_version(), "host": host_info(),
                   "side_kernels": side},
        "roofline": {"bound": "hbm", "achieved": round(hbm, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(hbm / HBM_PEAK_GBS, 4), "traffic": _pmc_traffic("k_copy"),
                     "kernel": "bine::k_copy (the P = 1 allreduce is one launch)",
                     "algorithmic_bytes_per_launch": 2 * S,
                     "us_per_launch": round(st_k["region_ms"] * 1e3, 3),
                     "note": "achieved = 2 S (read sbuf + write rbuf) / the average launch duration: K calls "
                             "(one k_copy launch each) back to back between one HIP event pair on the launch "
                             "stream (agrees with the kernel-trace average, profiles/r4_bench_kernel_stats.csv); "
                             "traffic = PMC FETCH_SIZE x 2 (gfx950) + WRITE_SIZE per launch "
                             "(profiles/latest_pmc.json)"},
        "wall_s": round(st["wall_s"], 4),
    }
    if want_cpu:
        out["cpu_baseline"] = cpu_baseline(dig, cpu_budget)
    return out


# ---- N > 1 ------------------------------------------------------------------------

BIT_EXACT_MARGIN = 1.03   # a bit-exact transport within 3 % of multi-tree mode is preferred


def _prefer_exact(times):
    """fastest transport of {mode: ms}; multi-tree mode (fp results within
    rounding of the reference, not bit-identical) only when it beats every
    bit-exact transport by more than BIT_EXACT_MARGIN"""
    best = min(times, key=times.get)
    exact = {m: t for m, t in times.items() if m != "trees"}
    if best == "trees" and exact:
        e = min(exact, key=exact.get)
        if exact[e] <= times[best] * BIT_EXACT_MARGIN:
            return e
    return best


def _side(rank, what, fn):
    """a side measurement beside the headline: its failure (a library error,
    symmetric on every rank since plans are a pure function of the arguments)
    is reported in the JSON line instead of ending the run"""
    try:
        return fn()
    except Exception as e:  # noqa: BLE001 -- reported, not swallowed
        if rank == 0:
            print(f"bench: {what} skipped: {e}", file=sys.stderr)
        return {"error": f"{type(e).__name__}: {e}"}


def overlap_frac(exchanges, locals_):
    """share of the local (reduction) time that runs while some exchange is in
    flight: sum over local ops of |local interval & union of exchange
    intervals| / sum of local durations; intervals are (start, duration)"""
    tot = sum(d for _, d in locals_)
    if tot <= 0:
        return None
    iv = sorted((s, s + d) for s, d in exchanges if d > 0)
    merged = []
    for a, b in iv:
        if merged and a <= merged[-1][1]:
            merged[-1][1] = max(merged[-1][1], b)
        else:
            merged.append([a, b])
    hid = 0.0
    for s, d in locals_:
        a, b = s, s + d
        hid += sum(max(0.0, min(b, y) - max(a, x)) for x, y in merged)
    return min(1.0, hid / tot)


def _step_profile(pico_amd, torch, dist, comm, algo, sbuf, rbuf, nelem, stream):
    return step_profile(torch, comm,
                        lambda: pico_amd.allreduce(algo, sbuf, rbuf, nelem, "float", "sum", comm, stream=stream),
                        dist)


def step_profile(torch, comm, call, dist=None):
    """One extra collective (outside the timed region) with per-op timing
    events (bine_comm_set_profile): where the time of this rank goes -- busy
    time of the comm stream (exchanges) and of the compute stream (reductions),
    their span, the share of the reductions' time during which an exchange
    is in flight (overlap_frac), and the exchange ops' egress rates."""
    comm.set_profile(True)
    d = Drain(comm)
    try:
        d.guard(call)()
        torch.cuda.synchronize()
        d()
        err = d.failed(dist)
        ops = comm.profile() if err is None else []
    finally:
        comm.set_profile(False)
    if err is not None:
        return {"error": err}
    if not ops:
        return {}
    span = max(o["start_ms"] + o["ms"] for o in ops)
    xs = [o for o in ops if o["xchg"]]
    ls = [o for o in ops if not o["xchg"]]
    lb_ops = [o for o in ls if o["nprims"]]   # nprims 0: a tree inside an exchange launch (no launch of its own)
    xb, lb = sum(o["ms"] for o in xs), sum(o["ms"] for o in lb_ops)
    ov = overlap_frac([(o["start_ms"], o["ms"]) for o in xs], [(o["start_ms"], o["ms"]) for o in lb_ops])
    return {"ops": len(ops), "span_ms": round(span, 4), "exchange_busy_ms": round(xb, 4),
            "local_busy_ms": round(lb, 4), "overlap_frac": None if ov is None else round(ov, 4),
            "exchanges": [{"start_ms": round(o["start_ms"], 4), "ms": round(o["ms"], 4), "peers": o["nprims"],
                           "egress_GBs": round(o["bytes"] / (o["ms"] * 1e-3) / 1e9, 2) if o["ms"] > 0 else None}
                          for o in xs[:24]],
            "local": [{"start_ms": round(o["start_ms"], 4), "ms": round(o["ms"], 4),
                       "hbm_GBs": round(o["bytes"] / (o["ms"] * 1e-3) / 1e9, 1) if o["ms"] > 0 and o["nprims"] else None}
                      | ({"inside_exchange": True} if not o["nprims"] else {})
                      for o in ls[:24]]}


def _dm_token(mode):
    i = mode.find("+dm")
    return None if i < 0 else mode[i + 3:].split("+")[0]


def dm_wgs(mode):
    """the direct transport's workgroups per message a mode names: "+dm" ->
    0 (the default, 128), "+dm64" / "+dmt64" / "+dmt64x128" -> 64; None when the
    mode does not use it"""
    tok = _dm_token(mode)
    if tok is None:
        return None
    digits = tok.lstrip("t").split("x")[0]
    return int(digits) if digits.isdigit() else 0


def dm_tree(mode):
    """the direct transport's fused trees (bine_comm_set_direct_tree) a mode
    names: "+dm" -> 0 (off: pull copies + a separate tree launch), "+dmt" ->
    1 (on, the default tree workgroups), "+dmtxT" / "+dmtWxT" -> T tree
    workgroups per launch"""
    tok = _dm_token(mode)
    if tok is None or not tok.startswith("t"):
        return 0
    t = tok.split("x")
    return int(t[1]) if len(t) > 1 and t[1].isdigit() else 1


def apply_transport(comm, mode, chunk, graphs=False):
    comm.set_graphs(graphs)
    w = dm_wgs(mode)
    comm.set_direct(w is not None)
    if w is not None:
        comm.set_direct_wgs(w)
        comm.set_direct_tree(dm_tree(mode))
    comm.set_relay(RELAY_MIN_BYTES if "relay" in mode else 0)
    comm.set_trees(mode.startswith("trees"))
    comm.set_flat_ag("flat" in mode)
    comm.set_flat_rs("flatrs" in mode)
    comm.set_coll_ag("+ag" in mode)
    comm.set_coll_a2a("+a2a" in mode)
    comm.set_chunk(chunk)


def _extra_configs(pico_amd, torch, dist, comm, stream, world, rank, dev, mode, chunk, graphs=False, dm_ok=False):
    """BASELINE configs C1, C4 and C5 on the transport chosen for C3 (C1: the
    bit-exact flat phases instead of multi-tree mode, a large-message mode;
    eager and graph-replayed), each checked against the oracle's digests of
    its inputs (seed 1234 + rank)"""
    out = {}
    # C1: fp32 allreduce 1 MiB per rank (the reference's own CPU configuration:
    # libbine bine_bdw_remap_over 381.9 us at P = 4 through pico_core,
    # BASELINE.md section 2) -- latency-bound: the bandwidth and the
    # latency-optimal Bine variants are both timed
    apply_transport(comm, "flatrs+flat" if mode == "trees" else mode, chunk, False)
    n1 = C1_ELEMS
    sb = torch.empty(n1, dtype=torch.float32, device=dev)
    rb = torch.empty(n1, dtype=torch.float32, device=dev)
    pico_amd.fill_pico(sb, n1, "float", 1234 + rank)
    for algo in ("bine_bdw_remap", "bine_lat"):
        for g in (False, True):   # eager issue, then the HIP-graph replay (bine_comm_set_graphs)
            comm.set_graphs(g)
            rb.fill_(float("nan"))
            st, err = measure(torch, stream, dist, comm,
                              lambda: pico_amd.allreduce(algo, sb, rb, n1, "float", "sum", comm, stream=stream),
                              50, 10)
            if err:
                out[f"C1_allreduce_{algo}_f32_1MiB" + ("_graph" if g else "")] = {"error": err}
                continue
            ok, _ = check_digest(pico_amd, rb, n1, "float", gkey("C1", "allreduce", algo, "float", n1, world), rank)
            out[f"C1_allreduce_{algo}_f32_1MiB" + ("_graph" if g else "")] = {
                "us": round(st["median_ms"] * 1e3, 2),
                "algbw_per_rank_GBs": round(n1 * 4 / (st["median_ms"] * 1e-3) / 1e9, 2),
                "host_issue_us": round(st["issue_ms"] * 1e3, 2), "parity_ok": all_ok(torch, dist, ok),
                **({"captured": comm.graphs_cached() > 0} if g else {})}
    comm.set_graphs(False)
    if dm_ok and "+dm" not in mode and world > 1:
        # C1 also over the direct peer-memory transport with the flat phases:
        # one k_dm_fused launch per call (the whole flat collective in one
        # kernel), beside the RCCL path chosen for C3
        try:
            apply_transport(comm, "flatrs+flat+dm", chunk, False)
            for algo in ("bine_bdw_remap", "bine_lat"):
                rb.fill_(float("nan"))
                st, err = measure(torch, stream, dist, comm,
                                  lambda: pico_amd.allreduce(algo, sb, rb, n1, "float", "sum", comm, stream=stream),
                                  50, 10)
                if err:
                    out[f"C1_allreduce_{algo}_f32_1MiB_direct_fused"] = {"error": err}
                    continue
                ok, _ = check_digest(pico_amd, rb, n1, "float", gkey("C1", "allreduce", algo, "float", n1, world),
                                     rank)
                out[f"C1_allreduce_{algo}_f32_1MiB_direct_fused"] = {
                    "us": round(st["median_ms"] * 1e3, 2),
                    "algbw_per_rank_GBs": round(n1 * 4 / (st["median_ms"] * 1e-3) / 1e9, 2),
                    "host_issue_us": round(st["issue_ms"] * 1e3, 2), "parity_ok": all_ok(torch, dist, ok)}
        except pico_amd.BineError as e:   # symmetric: setup is agreed over RCCL
            out["C1_direct_fused"] = {"error": str(e)}
    del sb, rb
    # C4 / C5 on the chosen transport, chunk and graph setting.  (Round 3 issued
    # them eagerly after a replay of the C4 reduce_scatter segfaulted inside
    # torch's HIP 7.0 under GPU_MAX_HW_QUEUES=1; the cause is that runtime's
    # Graph::UpdateStreams on graphs with parallel branches, and the library
    # now captures two-stream schedules only on HIP >= 7.2 --
    # profiles/r4_graph_fork_repro.txt.)
    apply_transport(comm, mode, chunk, graphs)
    trees = mode == "trees"
    # C4: reduce_scatter_bine_permute_remap fp32, 1 GiB input per rank
    n = C4_ELEMS
    sb = torch.empty(n, dtype=torch.float32, device=dev)
    rb = torch.empty(n // world, dtype=torch.float32, device=dev)
    pico_amd.fill_pico(sb, n, "float", 1234 + rank)
    rc = [n // world] * world
    st, err = measure(torch, stream, dist, comm,
                      lambda: pico_amd.reduce_scatter("bine_permute_remap", sb, rb, rc, "float", "sum", comm,
                                                      stream=stream),
                      5, 2)
    ok, _ = check_digest(pico_amd, rb, n // world, "float",
                         gkey("C4", "reduce_scatter", "bine_permute_remap", "float", n, world, trees), rank)
    S = n * 4
    nm = node_model("C4", world, mode, chunk)
    c4 = "C4_reduce_scatter_bine_permute_remap_f32_1GiB"
    out[c4] = {"error": err} if err else {
        "ms": round(st["median_ms"], 4),
        "busbw_per_rank_GBs": round((world - 1) / world * S / (st["median_ms"] * 1e-3) / 1e9, 2),
        "graph_replay": graphs and comm.graphs_cached() > 0, "parity_ok": all_ok(torch, dist, ok),
        "model_ms": nm.get("model_ms"),
        "frac_of_model": round(nm["model_ms"] / st["median_ms"], 4) if nm.get("model_ms") else None}
    del sb, rb
    # C5: allreduce_bine_bdw_remap fp64 / int64 SUM, 256 MiB per rank
    n = C5_ELEMS
    for dt, tdt in (("double", torch.float64), ("int64", torch.int64)):
        if graphs:   # an empty graph cache: graphs_cached() below is this configuration's
            comm.set_graphs(False)
            comm.set_graphs(True)
        sb = torch.empty(n, dtype=tdt, device=dev)
        rb = torch.empty(n, dtype=tdt, device=dev)
        pico_amd.fill_pico(sb, n, dt, 1234 + rank)
        st, err = measure(torch, stream, dist, comm,
                          lambda: pico_amd.allreduce("bine_bdw_remap", sb, rb, n, dt, "sum", comm, stream=stream),
                          5, 2)
        if err:
            out[f"C5_allreduce_bine_bdw_remap_{dt}_256MiB"] = {"error": err}
            del sb, rb
            continue
        ok, _ = check_digest(pico_amd, rb, n, dt, gkey("C5", "allreduce", "bine_bdw_remap", dt, n, world, trees), rank)
        S = n * 8
        ms = st["median_ms"]
        nm = node_model("C5", world, mode, chunk)
        out[f"C5_allreduce_bine_bdw_remap_{dt}_256MiB"] = {
            "ms": round(ms, 4), "algbw_per_rank_GBs": round(S / (ms * 1e-3) / 1e9, 2),
            "busbw_per_rank_GBs": round(2 * (world - 1) / world * S / (ms * 1e-3) / 1e9, 2),
            "graph_replay": graphs and comm.graphs_cached() > 0, "parity_ok": all_ok(torch, dist, ok),
            "model_ms": nm.get("model_ms"), "frac_of_model": round(nm["model_ms"] / ms, 4) if nm.get("model_ms") else None}
        del sb, rb
    torch.cuda.empty_cache()
    return out


def _p2p_probe(pico_amd, torch, dist, comm, stream, world, rank, dev, per_peer=32 << 20):
    """RCCL P2P calibration of this node through the same transport the
    collectives use (bine_exchange = one ncclGroupStart/End): (a) one peer,
    rank r <-> r^1 both ways; (b) all P-1 peers at once (what relay / trees
    modes do per step).  GB/s per rank and direction."""
    out = {"bytes_per_peer": per_peer}
    comm.set_direct(False)   # the probe measures RCCL's own point-to-point path
    sb = torch.empty(per_peer * (world - 1), dtype=torch.uint8, device=dev)
    rb = torch.empty(per_peer * (world - 1), dtype=torch.uint8, device=dev)
    sb.fill_(rank & 0xFF)
    torch.cuda.synchronize()
    if world % 2 == 0:
        peer = rank ^ 1
        st = timed(torch, stream,
                   lambda: pico_amd.exchange(comm, [(peer, sb, per_peer)], [(peer, rb, per_peer)], stream=stream),
                   10, 3, dist, (comm.synchronize,))
        out["one_peer_GBs"] = round(per_peer / (st["median_ms"] * 1e-3) / 1e9, 2)
    peers = [p for p in range(world) if p != rank]
    sends = [(p, sb[i * per_peer:], per_peer) for i, p in enumerate(peers)]
    recvs = [(p, rb[i * per_peer:], per_peer) for i, p in enumerate(peers)]
    st = timed(torch, stream, lambda: pico_amd.exchange(comm, sends, recvs, stream=stream), 10, 3, dist,
               (comm.synchronize,))
    out["all_peers_egress_GBs"] = round(len(peers) * per_peer / (st["median_ms"] * 1e-3) / 1e9, 2)
    del sb, rb
    torch.cuda.empty_cache()
    return out


def _direct_probe(pico_amd, torch, dist, comm, stream, world, rank, dev, iters=1000, nbytes=64 << 20):
    """The two node constants the model assumes for the direct transport,
    measured per peer pair: the cross-GPU flag round trip
    (bine_comm_direct_ping: `iters` round trips inside one launch per side,
    the transport's own store / poll protocol) and the one-link push rate (a
    `nbytes` exchange with that peer alone, both directions at once, over the
    direct transport).  Pairs in the rounds of a 1-factorisation: rank r with
    r xor k, k = 1 .. P'-1 (P' the next power of two; a rank whose partner
    does not exist sits the round out).  Rank 0 gets every pair's values,
    their medians and the model's constants beside them."""
    from pico_amd import model as NM
    apply_transport(comm, "direct+dm", nbytes)
    sb = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    rb = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    sb.fill_(rank & 0xFF)
    torch.cuda.synchronize()
    rtt, gbs, errs = {}, {}, []
    p2 = 1 << (world - 1).bit_length()
    for k in range(1, p2):
        peer = rank ^ k
        if peer < world:
            try:
                rtt[peer] = comm.direct_ping(peer, iters)
            except pico_amd.BineError as e:
                errs.append(f"ping {rank}-{peer}: {e}")
        call = (lambda p=peer: pico_amd.exchange(comm, [(p, sb, nbytes)], [(p, rb, nbytes)], stream=stream)) \
            if peer < world else (lambda: None)
        st, err = measure(torch, stream, dist, comm, call, 10, 3)   # every rank: the same barriers
        if err:
            errs.append(f"push {rank}-{peer}: {err}")
        elif peer < world:
            gbs[peer] = nbytes / (st["median_ms"] * 1e-3) / 1e9
    del sb, rb
    torch.cuda.empty_cache()
    allv = [None] * world
    dist.all_gather_object(allv, (rtt, gbs, errs))
    pr = {f"{r}-{p}": round(v, 3) for r, (t, _, _) in enumerate(allv) for p, v in t.items() if r < p}
    pg = {f"{r}-{p}": round(v, 2) for r, (_, g, _) in enumerate(allv) for p, v in g.items()}
    out = {"flag_round_trip_us": pr, "push_GBs": pg, "push_bytes": nbytes, "ping_iters": iters,
           "errors": [e for _, _, es in allv for e in es][:8],
           "model_T_FLAG_US": NM.T_FLAG_US, "model_LINK_GBS": NM.LINK_GBS}
    if pr:
        out["flag_round_trip_us_median"] = round(statistics.median(pr.values()), 3)
        out["flag_one_way_us_median"] = round(statistics.median(pr.values()) / 2, 3)
    if pg:
        out["push_GBs_median"] = round(statistics.median(pg.values()), 2)
    return out


def _vendor_allreduce(pico_amd, torch, dist, comm, sbuf, rbuf, nelem, stream, world, bine_ms):
    """RCCL's own ncclAllReduce (fp32 SUM) on the same communicator, buffers and
    stream: the vendor collective the Bine path competes with on this node.
    Its reduction order is RCCL's, not the reference's (a baseline, not a
    libbine result)."""
    st = timed(torch, stream,
               lambda: pico_amd.vendor_allreduce(sbuf, rbuf, nelem, "float", "sum", comm, stream=stream),
               10, 3, dist, (comm.synchronize,))
    ms = st["median_ms"]
    S = nelem * 4
    return {"ms": round(ms, 4), "algbw_per_rank_GBs": round(S / (ms * 1e-3) / 1e9, 2),
            "busbw_per_rank_GBs": round(2 * (world - 1) / world * S / (ms * 1e-3) / 1e9, 2),
            "bine_speedup": round(ms / bine_ms, 3)}


RELAY_MIN_BYTES = 256 << 10    # smallest relayed part when relay mode is on
DM_WGS_TRIALS = (64, 256)      # direct transport: workgroups per message tried beside the default 128
TREE_WGS_TRIALS = (512, 1024)  # fused trees ("+dmt"): tree workgroups per launch tried beside the default 256
#                               (a large flat call as one k_dm_fused launch: its whole grid)
CHUNK_TRIALS = (4 << 20, 8 << 20, 16 << 20, 32 << 20, 64 << 20)   # pipelining chunks tried at N > 1
MODES = {"off": ["direct"],
         # "+a2a" is not tried: RCCL runs ncclAllToAllv as the same grouped P2P kernel
         # (rcclGenericKernel) as P-1 ncclSend/ncclRecv pairs (profiles/r2_a2a_vs_p2p_kernels.txt)
         # "+dm": the direct peer-memory transport (bine_comm_set_direct) instead of RCCL;
         # "+dmt": the same with the flat reduce-scatter's trees inside its exchange
         # launches (bine_comm_set_direct_tree: no pull copies of the leaves)
         "auto": ["direct", "flat", "relay", "relay+flat", "flatrs+flat", "flatrs+flat+ag", "trees",
                  "direct+dm", "flatrs+flat+dm", "flatrs+flat+dmt", "relay+flat+dm"]}


def node_model(cfg, world, mode, chunk):
    """pico_amd.model's expected time of BASELINE config `cfg` on this node for
    transport `mode` (its workgroup suffixes dropped) at pipelining chunk
    `chunk`: max(link time, HBM time) + launches x boundary; with
    BINE_FAKE_HOSTS (several ranks on one GPU) the one-GPU form (every rank's
    bytes through one HBM, no link)"""
    try:
        from pico_amd import model as NM
        t = re.sub(r"(\+dmt?)\d*(x\d+)?", r"\1", mode)
        m = NM.config_model(cfg, world, t, chunk, one_gpu=os.environ.get("BINE_FAKE_HOSTS") == "1")
        m.update(link_GBs=NM.LINK_GBS, hbm_rate_GBs=NM.HBM_RATE_GBS, boundary_us=NM.T_BOUNDARY_US,
                 one_gpu=os.environ.get("BINE_FAKE_HOSTS") == "1")
        return m
    except Exception as e:  # the model is a report, never a reason to lose the line
        return {"error": str(e)}


def measured_models(world, mode, chunk, link_gbs, t_flag_us):
    """pico_amd.model's C3 / C4 / C5 expectation for `mode` with the measured
    link rate, and the C1 end-to-end expectation with the measured per-phase
    flag latency (bench.py's direct-transport probe); the one-GPU form when
    ranks share a GPU (then no link: the values say what the probe saw)"""
    try:
        from pico_amd import model as NM
        t = re.sub(r"(\+dmt?)\d*(x\d+)?", r"\1", mode)
        one = os.environ.get("BINE_FAKE_HOSTS") == "1"
        res = {"link_GBs": link_gbs, "t_flag_us": t_flag_us, "one_gpu": one}
        for cfg in ("C3", "C4", "C5"):
            res[cfg] = NM.config_model(cfg, world, t, chunk, one_gpu=one, link_gbs=link_gbs)["model_ms"]
        if t_flag_us is not None:
            # ranks sharing one GPU: the push figure is no link rate (DESIGN.md
            # 7.2), so the node's C1 takes the measured flag latency with the
            # model's link rate
            res["C1_e2e_us"] = NM.c1_e2e_us(world, t_flag_us=t_flag_us,
                                            link_gbs=NM.LINK_GBS if one else link_gbs)["e2e_us"]
            if one:
                res["C1_note"] = "one GPU: C1_e2e_us = the node model with the measured flag latency and the assumed link rate"
        return res
    except Exception as e:  # a report, never a reason to lose the line
        return {"error": str(e)}


def transport_modes(relay: str, world: int):
    """transports: "direct" = the literal Bine schedule (one peer per step);
    "relay" = the same schedule with permutation steps routed over all links
    (two hops); "+flat" = the allgather phase as one all-peers exchange (one
    hop on every link); "flatrs" = the reduce-scatter phase as one all-peers
    exchange whose owner evaluates the reference's reduction tree in one fused
    kernel; "+ag" / "+a2a" = the flat exchanges as ncclAllGather /
    ncclAllToAllv; "+dm" = exchanges through mapped peer memory instead of
    RCCL; "trees" = P-1 relabelled instances over edge-disjoint pairings.
    All but "trees" are bit-identical to the reference."""
    modes = MODES.get(relay, [relay])
    if world <= 2:
        modes = [m for m in modes if "relay" not in m and "+ag" not in m and "+a2a" not in m] or ["direct"]
    if world not in (4, 8):
        modes = [m for m in modes if not m.startswith("trees")] or ["direct"]
    if world & (world - 1):
        modes = [m for m in modes if "flat" not in m] or ["direct"]
    return modes


def link_roofline(pico_amd, algo, world, rank, nelem, chunk, chosen):
    """bytes this rank puts on xGMI per allreduce (executed schedule) and the
    schedule-aware link bound: exchange ops run one after another, the links
    of one op in parallel, so at B GB/s per link the schedule needs at least
    L / B, L = sum over ops of the busiest link's bytes"""
    ops, _, _ = pico_amd.schedule("allreduce", algo, world, rank, count=nelem, esz=4, chunk_bytes=chunk,
                                  relay_min_bytes=RELAY_MIN_BYTES if "relay" in chosen else 0,
                                  trees=chosen == "trees", flat_ag="flat" in chosen, flat_rs="flatrs" in chosen)
    egress = 4 * sum(p["count"] for o in ops if o["xchg"] for p in o["prims"] if p["type"] == "SEND")
    peers = len({p["peer"] for o in ops if o["xchg"] for p in o["prims"] if p["type"] == "SEND"})
    L = 0
    op_links = []  # per exchange op: (busiest directed link's bytes, peers it talks to)
    for o in ops:
        if o["xchg"]:
            lk = {}
            for p in o["prims"]:
                if p["type"] in ("SEND", "RECV"):
                    lk[(p["type"], p["peer"])] = lk.get((p["type"], p["peer"]), 0) + 4 * p["count"]
            L += max(lk.values())
            op_links.append((max(lk.values()), len({p["peer"] for p in o["prims"]})))
    return egress, peers, L, op_links


def tname(cfg):
    """trial label: transport/chunk[+sK][+graph]"""
    return f"{cfg[0]}/{cfg[1] >> 20}MiB" + ("+graph" if len(cfg) > 2 and cfg[2] else "")


def _best_of(trials, verdicts, nbytes, keep):
    """the fastest trial config passing `keep` whose output matched the
    oracle: {transport, ms, algbw_per_rank_GBs} (None if there is none)"""
    ok = [(v, c) for c, v in trials.items() if keep(c) and verdicts.get(c) is True and v != float("inf")]
    if not ok:
        return None
    v, c = min(ok)
    return {"transport": tname(c), "ms": round(v, 4), "algbw_per_rank_GBs": round(nbytes / (v * 1e-3) / 1e9, 2)}


DEADLINE_EXIT = 3   # exit status of a run cut by a deadline (its JSON line says "cut_by_deadline")


def arm_deadline(budget_s, payload, what):
    """A daemon timer: unless cancelled within budget_s seconds, print
    payload() as the JSON line (when it is not None -- rank 0) marked
    "cut_by_deadline": <what>, say so on stderr and end the process with
    status DEADLINE_EXIT, so that a hang is never mistaken for a clean run.
    Every rank arms the same budget, so all ranks stop together instead of
    waiting in a collective a hung peer never joins.  (os._exit: no re-exec,
    nothing restarts a process that has touched the GPU.)"""
    def fire():
        line = payload()
        if line is not None:
            line["cut_by_deadline"] = what
            print(json.dumps(line), flush=True)
        sys.stderr.write(f"bench: {what} exceeded {budget_s:.0f} s; exiting with status {DEADLINE_EXIT}\n")
        sys.stderr.flush()
        os._exit(DEADLINE_EXIT)

    t = threading.Timer(budget_s, fire)
    t.daemon = True
    t.start()
    return t


def bench_allreduce(steps: int, warmup: int, nelem: int, algo: str, relay: str, extras: bool = True,
                    chunk_mib: int = 0, graph_trial: bool = True):
    import pico_amd
    import torch
    import torch.distributed as dist
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    local = int(os.environ.get("LOCAL_RANK", rank))
    if os.environ.get("BINE_FAKE_HOSTS") == "1":
        # rehearsal with several ranks on one GPU: RCCL needs distinct host ids
        # (socket transport on lo; says nothing about xGMI speed)
        os.environ["NCCL_HOSTID"] = f"bine-fake-host-{rank}"
        os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")
    local %= torch.cuda.device_count()
    torch.cuda.set_device(local)
    dist.init_process_group("gloo")
    with quiet_stdout():
        comm = pico_amd.Comm.from_torch_distributed(local)
    dev = torch.device("cuda", local)
    # one non-NULL stream for everything (torch ops, fills, checksums and the
    # collectives): graph mode cannot capture the legacy NULL stream
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    sbuf = torch.empty(nelem, dtype=torch.float32, device=dev)
    rbuf = torch.empty(nelem, dtype=torch.float32, device=dev)
    pico_amd.fill_pico(sbuf, nelem, "float", 1234 + rank)
    torch.cuda.synchronize()
    modes = transport_modes(relay, world)
    chunks = [chunk_mib << 20] if chunk_mib else list(CHUNK_TRIALS)
    key = gkey("C3", "allreduce", algo, "float", nelem, world)
    key_trees = gkey("C3", "allreduce", algo, "float", nelem, world, True)

    def run():
        pico_amd.allreduce(algo, sbuf, rbuf, nelem, "float", "sum", comm, stream=stream)

    def parity(mode):
        ok, d = check_digest(pico_amd, rbuf, nelem, "float", key_trees if mode.startswith("trees") else key, rank,
                             stream)
        return all_ok(torch, dist, ok), d

    # measured, not guessed: each transport is timed briefly on this hardware
    # (max over ranks, so every rank picks the same) and its output checked
    # against the oracle's digest; then the pipelining chunk for the fastest
    # correct one; the fastest pair is kept
    trials, verdicts = {}, {}

    dm_dead = []   # the direct transport could not be set up: not tried again (a timed-out wait is not
    #                this: the next bine_comm_set_direct(1) rebuilds the transport on every rank)

    def trial(cfg):
        # a setting the planner rejects fails identically on every rank before
        # any transfer (plans are a pure function of the arguments): skip it
        cfg = tuple(cfg) + (False,)[len(cfg) - 2:]
        if dm_dead and dm_wgs(cfg[0]) is not None:
            trials[cfg] = float("inf")
            verdicts[cfg] = "error"
            return
        try:
            # inside: enabling the direct transport fails on every rank alike
            # when peer memory cannot be mapped (BINE_ERR_UNSUPPORTED)
            if cfg[2]:
                comm.set_graphs(False)   # an empty graph cache: graphs_cached() then says whether this one captured
            apply_transport(comm, *cfg)
            rbuf.fill_(float("nan"))   # a transport that writes nothing cannot pass on the last one's output
            st, why_err = measure(torch, stream, dist, comm, run, 3, 2)
            ok, _ = parity(cfg[0])
            # a call whose direct-transport wait timed out reports it at its
            # completion on the rank that timed out (the call ran on without
            # its data): agreed over the ranks, with the waiter's record
            verdicts[cfg] = ok if why_err is None else f"failed: {why_err}"[:16000]
            trials[cfg] = st["median_ms"] if ok is not False and why_err is None else float("inf")
            if cfg[2] and comm.graphs_cached() == 0:
                # the library kept every call eager (its HIP-runtime gate,
                # include/bine_amd.h): not a graph replay, so not picked as one
                verdicts[cfg] = "eager (not captured)"
                trials[cfg] = float("inf")
            if (ok is False or why_err is not None) and rank == 0:
                why = why_err or "output digest differs from the oracle's"
                print(f"bench: transport {tname(cfg)} EXCLUDED: {why}", file=sys.stderr)
        except pico_amd.BineError as e:
            if rank == 0:
                print(f"bench: transport {tname(cfg)} skipped: {e}", file=sys.stderr)
            torch.cuda.synchronize()
            Drain(comm)()
            trials[cfg] = float("inf")
            verdicts[cfg] = f"error: {e}"[:2000]
            if dm_wgs(cfg[0]) is not None and e.status == 6:   # BINE_ERR_UNSUPPORTED: setup failed
                # symmetric: setup is agreed over RCCL, so every rank stops
                # trying together
                dm_dead.append(tname(cfg))

    mid = 16 << 20 if 16 << 20 in chunks else chunks[0]
    S = nelem * 4

    def headline(cfg, st, ok_head, dig, ok_trees_tol=None):
        """rank 0's JSON line for a timed, checked configuration (None elsewhere)"""
        if rank != 0:
            return None
        return _headline_line(pico_amd, algo, world, rank, nelem, steps, warmup, key, cfg, st, ok_head, dig,
                              ok_trees_tol, trials, verdicts)

    # A provisional line first: the literal Bine schedule over RCCL P2P (the
    # path every test exercises) timed in full and checked.  The trials below
    # then run under a deadline: should one of them hang inside RCCL or the
    # direct transport on the driver's node (configurations no one-GPU box can
    # rehearse over xGMI), every rank stops at the same budget and rank 0
    # prints this line instead of losing the run.
    base_cfg = ("direct", mid, False)
    apply_transport(comm, *base_cfg)
    rbuf.fill_(float("nan"))
    st0 = timed(torch, stream, run, steps, warmup, dist, (comm.synchronize,))
    ok0, dig0 = parity("direct")
    provisional = headline(base_cfg, st0, ok0, dig0)
    trial_budget = float(os.environ.get("BENCH_TRIAL_BUDGET_S", "180"))

    def _provisional():
        if provisional is not None:
            provisional["config"]["transport_trials_cut_after_s"] = trial_budget
            provisional["config"]["transport_trials_ms"] = {tname(c): round(v, 4) for c, v in trials.items()}
            provisional["config"]["parity"]["trials"] = {tname(c): v for c, v in verdicts.items()}
        return provisional

    watchdog = arm_deadline(trial_budget, _provisional, "transport trials")
    if len(modes) > 1 or len(chunks) > 1:
        for m in modes:
            trial((m, mid, False))
        finite = {c[0]: v for c, v in trials.items() if c[1] == mid and v != float("inf")}
        m_best = _prefer_exact(finite) if finite else "direct"
        for ch in chunks:
            if (m_best, ch, False) not in trials:
                trial((m_best, ch, False))
        cands = [c for c in trials if c[0] == m_best and trials[c] != float("inf")]
        best = min(cands, key=trials.get) if cands else base_cfg
        if dm_wgs(best[0]) == 0:
            # the direct transport's workgroups per message at the chosen chunk
            # (default 128): how many it takes to fill a link is the node's to say
            for w in DM_WGS_TRIALS:
                trial((best[0] + str(w), best[1], False))
            cands = [c for c in trials if c[1] == best[1] and not c[2] and trials[c] != float("inf")
                     and (c[0] == best[0] or c[0] in [best[0] + str(w) for w in DM_WGS_TRIALS])]
            best = min(cands, key=trials.get)
        if dm_tree(best[0]) == 1:
            # the fused trees' workgroups per launch (default 256): on a node each
            # GPU's CUs serve one rank, so more of them may pay there
            names = [best[0] + "x" + str(t) for t in TREE_WGS_TRIALS]
            for nm in names:
                trial((nm, best[1], False))
            cands = [c for c in trials if c[1] == best[1] and not c[2] and trials[c] != float("inf")
                     and (c[0] == best[0] or c[0] in names)]
            best = min(cands, key=trials.get)
    else:
        best = (modes[0], chunks[0], False)
    if graph_trial:
        # the same transport x chunk issued as one HIP-graph replay per call
        trial((best[0], best[1], True))
        if trials[(best[0], best[1], True)] < trials.get(best, float("inf")):
            best = (best[0], best[1], True)
    if dm_dead and dm_wgs(best[0]) is not None:
        # a direct transport that could not be set up in a later trial: the
        # pick falls back to the fastest checked setting without it
        ok_c = [c for c, v in trials.items() if v != float("inf") and dm_wgs(c[0]) is None]
        best = min(ok_c, key=trials.get) if ok_c else base_cfg
        if rank == 0:
            print(f"bench: the direct transport failed in trial {dm_dead[0]}; picking {tname(best)}", file=sys.stderr)
    def full_run(cfg):
        """(stats, ok, digest) of a full timed run of cfg; a library error
        (e.g. a direct-transport wait that timed out: BINE_ERR_INTERNAL on the
        next call) is a failed check, never the end of the bench"""
        try:
            apply_transport(comm, *cfg)
            rbuf.fill_(float("nan"))
            st_, why_err = measure(torch, stream, dist, comm, run, steps, warmup)
            ok_, dig_ = parity(cfg[0])
            if why_err is not None:
                if rank == 0:
                    print(f"bench: {tname(cfg)} failed in its full run: {why_err}", file=sys.stderr)
                return ({"median_ms": float("inf")}, False, None)
            return st_, ok_, dig_
        except pico_amd.BineError as e:
            if rank == 0:
                print(f"bench: {tname(cfg)} failed in its full run: {e}", file=sys.stderr)
            torch.cuda.synchronize()
            return ({"median_ms": float("inf")}, False, None)

    run1 = None
    if best != base_cfg:
        run1 = full_run(best)
        st1 = run1[0]
        if rank == 0 and (run1[1] is False or run1[0]["median_ms"] >= st0["median_ms"]):
            print(f"bench: the trials' pick {tname(best)} timed in full: {run1[0]['median_ms']:.4f} ms, parity "
                  f"{run1[1]}" + (" (a direct-transport wait timed out)" if dm_wgs(best[0]) is not None and
                                  comm.direct_timed_out() else "") + f"; the literal schedule: "
                  f"{st0['median_ms']:.4f} ms", file=sys.stderr)
        if run1[1] is False:
            # the pick failed its check in full: one full run of the runner-up
            # (the fastest other checked trial) before the literal schedule
            nxt = runner_up(trials, best, base_cfg)
            if nxt is not None:
                best = nxt
                run1 = full_run(best)
                st1 = run1[0]
                if rank == 0:
                    print(f"bench: runner-up {tname(best)} timed in full: {st1['median_ms']:.4f} ms, parity "
                          f"{run1[1]}", file=sys.stderr)
    best, (st, ok_head, dig) = pick_headline(base_cfg, (st0, ok0, dig0), best, run1)
    chosen, chunk, graphs = best
    apply_transport(comm, chosen, chunk, graphs)
    ok_trees_tol = None
    if chosen == "trees":
        # fp results of multi-tree mode are the reference's schedule on
        # relabelled ranks: checked exactly against that (digest above) and
        # against the reference's own bits with pico_core's ground-truth
        # tolerance (pico_core_utils.c:960-992: |a - b| <= P * 1e-6 * 100)
        run()
        torch.cuda.synchronize()
        tree_out = rbuf.clone()
        apply_transport(comm, "flatrs+flat", chunk, graphs)
        run()
        torch.cuda.synchronize()
        ok_exact, _ = parity("flatrs+flat")
        tol = world * 1e-6 * 100.0
        ok_trees_tol = all_ok(torch, dist, bool(ok_exact) and float((tree_out - rbuf).abs().max()) <= tol)
        del tree_out
        apply_transport(comm, chosen, chunk, graphs)
    watchdog.cancel()
    ms = st["median_ms"]
    out = headline(best, st, ok_head, dig, ok_trees_tol)
    # the side measurements below run under a deadline: if one of them hangs
    # (an RCCL or transport fault in a secondary configuration), every rank
    # stops at the same budget and rank 0 still prints the headline line with
    # what was measured so far -- a hang after the headline must not lose it
    budget = float(os.environ.get("BENCH_SIDE_BUDGET_S", "180"))

    def _partial():
        if out is not None:
            out["config"]["side_measurements_cut_after_s"] = budget
        return out

    watchdog = arm_deadline(budget, _partial, "side measurements")
    if rank == 0:
        print(f"bench: headline {tname(best)} {ms:.4f} ms; side measurements next", file=sys.stderr, flush=True)
    steps_prof = _side(rank, "step profile", lambda: _step_profile(pico_amd, torch, dist, comm, algo, sbuf, rbuf, nelem,
                                                                      stream))
    extra = _side(rank, "C1/C4/C5", lambda: _extra_configs(pico_amd, torch, dist, comm, stream, world, rank, dev,
                                                           chosen, chunk, graphs, not dm_dead)) if extras else {}
    try:
        apply_transport(comm, chosen, chunk, graphs)
    except pico_amd.BineError as e:   # the direct transport timed out in a side measurement: RCCL from here on
        if rank == 0:
            print(f"bench: {tname(best)} unavailable after the side measurements ({e}); RCCL P2P for the rest",
                  file=sys.stderr)
        apply_transport(comm, "direct", chunk, False)
    # the direct transport's flag round trip and one-link push rate per peer
    # pair: the node model's two assumed constants, measured
    dprobe = _side(rank, "direct-transport probe",
                   lambda: _direct_probe(pico_amd, torch, dist, comm, stream, world, rank, dev)) \
        if extras and not dm_dead else {}
    probe = _side(rank, "P2P probe", lambda: _p2p_probe(pico_amd, torch, dist, comm, stream, world, rank, dev)) \
        if extras else {}
    vendor = _side(rank, "RCCL allreduce", lambda: _vendor_allreduce(pico_amd, torch, dist, comm, sbuf, rbuf, nelem,
                                                                      stream, world, ms)) if extras else {}
    watchdog.cancel()
    if out is not None:
        out["config"].update({"step_profile_rank0": steps_prof, "other_baseline_configs": extra,
                              "rccl_p2p_probe": probe, "rccl_allreduce_baseline": vendor,
                              "direct_transport_probe": dprobe,
                              "transport_trials_ms": {tname(c): round(v, 4) for c, v in trials.items()},
                              "provisional_literal_rccl": {"ms": round(st0["median_ms"], 4),
                                                           "algbw_per_rank_GBs": round(S / (st0["median_ms"] * 1e-3) / 1e9, 2),
                                                           "parity_ok": ok0}})
        out["config"]["parity"]["trials"] = {tname(c): v for c, v in verdicts.items()}
    if rank == 0 and dprobe.get("push_GBs_median"):
        # the node model again with the measured constants in place of the
        # assumed ones: the link rate (C3 / C4 / C5) and the per-phase flag
        # latency of the C1 end-to-end model (one way = round trip / 2)
        out["roofline"]["model_with_measured_constants"] = measured_models(
            world, chosen, chunk, dprobe["push_GBs_median"], dprobe.get("flag_one_way_us_median"))
    if rank == 0:
        # the same egress against what RCCL P2P itself moves on this node: per
        # exchange op its busiest link at what RCCL moves per link in that
        # pattern -- the one-peer rate for a one-peer op, the all-peers egress
        # rate / (P - 1) when the op talks to several peers at once
        one, allp = probe.get("one_peer_GBs"), probe.get("all_peers_egress_GBs")
        lroof = out["roofline"].get("link_roofline_if_node", out["roofline"])
        L = lroof["link_time_bytes"]
        if one and L:
            op_links = link_roofline(pico_amd, algo, world, rank, nelem, chunk, chosen)[3]
            per_link_all = min(one, allp / (world - 1)) if allp else one
            t_rccl = sum(b / ((one if npeers <= 1 else per_link_all) * 1e9) for b, npeers in op_links)
            lroof["rccl_p2p_one_link_GBs"] = one
            lroof["rccl_p2p_per_link_all_peers_GBs"] = round(per_link_all, 2)
            lroof["frac_of_rccl_p2p_bound"] = round(t_rccl / (ms * 1e-3), 4)
    comm.destroy()
    dist.destroy_process_group()
    return out


def runner_up(trials, best, base):
    """the fastest checked trial other than the failed pick and the literal
    schedule (None when there is none)"""
    rest = [c for c, v in trials.items() if v != float("inf") and c not in (best, base)]
    return min(rest, key=trials.get) if rest else None


def pick_headline(base, run0, best, run1):
    """the headline among two full, checked runs (st, ok, digest): the
    provisional literal schedule `base` and the trials' pick `best` (run1 None
    when that is the same configuration).  A run whose check failed never wins
    over one that did not; otherwise the faster median wins (the trials'
    3-step estimates can mislead, the provisional run is a measurement too)."""
    if run1 is None:
        return base, run0
    ok0, ok1 = run0[1], run1[1]
    if (ok1 is False) != (ok0 is False):
        return (base, run0) if ok1 is False else (best, run1)
    return (base, run0) if run0[0]["median_ms"] < run1[0]["median_ms"] else (best, run1)


def _headline_line(pico_amd, algo, world, rank, nelem, steps, warmup, key, cfg, st, ok_head, dig, ok_trees_tol,
                   trials, verdicts):
    """the N > 1 JSON line for one timed configuration cfg = (transport, chunk,
    graphs): per-rank algbw, busbw, schedule-aware link roofline"""
    chosen, chunk, graphs = cfg
    ms = st["median_ms"]
    S = nelem * 4
    algbw = S / (ms * 1e-3) / 1e9
    busbw = 2 * (world - 1) / world * S / (ms * 1e-3) / 1e9
    egress, peers, L, _ = link_roofline(pico_amd, algo, world, rank, nelem, chunk, chosen)
    # schedule-aware link roofline: peak = the egress rate the schedule's link
    # time allows at 153 GB/s per link (153 for the literal one-peer-per-step
    # schedule, up to 7 x 153 when every step loads all links)
    link_peak = round(XGMI_LINK_GBS * egress / L, 2) if L else XGMI_LINK_GBS
    achieved = egress / (ms * 1e-3) / 1e9   # the headline statistic (median), as value and ms_per_step
    nm = node_model("C3", world, chosen, chunk) if nelem == C3_ELEMS and algo == "bine_bdw_remap" else {}
    out = {
        "metric": METRIC, "value": round(algbw, 2), "unit": "GB/s", "n_gpus": world, "steps": steps,
        "warmup": warmup, "ms_per_step": round(ms, 4), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "f32",
        "data": "synthetic (pico_core rand_r distribution, seed 1234 + rank, generated on device)",
        "config": {"workload": f"C3: allreduce_{algo} fp32 SUM {S // MIB} MiB/rank over "
                               f"{'mapped peer memory' if '+dm' in chosen else 'RCCL P2P'} (xGMI), "
                               f"{world} x MI355X, device-resident",
                   "value_definition": "per-rank algbw = S / t, t = per-iteration max over ranks, median after "
                                       "dropping the first 20 % (pico_core.c:133-140, summarize_data.py:24-48)",
                   "stats_ms": {k: _r(v, 5) for k, v in st.items()},
                   "algbw_per_rank_GBs": round(algbw, 2), "busbw_per_rank_GBs": round(busbw, 2),
                   "whole_job_GBs": round(world * algbw, 2),
                   "busbw_frac_of_target_1071": round(busbw / TARGET_BUSBW_GBS, 4),
                   "transport": chosen, "graph_replay": graphs,
                   "bit_exact_vs_reference": chosen != "trees" or "integers only (fp: within rounding)",
                   "chunk_bytes": chunk,
                   "parity": {"headline_ok": ok_head, "digest": str(dig),
                              "check": f"bine_checksum(rbuf) on every rank == oracle digest {key}"
                                       + (" (trees: relabelled-schedule digest)" if chosen == "trees" else ""),
                              "trees_within_pico_core_eps": ok_trees_tol,
                              "trials": {tname(c): v for c, v in verdicts.items()}},
                   "host_issue_ms_per_step": round(st["issue_ms"], 4),
                   "step_profile_rank0": None,
                   "transport_trials_ms": {tname(c): round(v, 4) for c, v in trials.items()},
                   # north_star names RCCL point-to-point: the fastest correct
                   # RCCL transport's figure beside the headline, whichever won
                   "best_rccl_p2p": _best_of(trials, verdicts, S, lambda c: "+dm" not in c[0]),
                   "xgmi_egress_bytes_per_rank": egress, "peers_per_rank": peers,
                   "other_baseline_configs": None,
                   "rccl_p2p_probe": None,
                   "rccl_allreduce_baseline": None,
                   "rccl": pico_amd.rccl_version(), "host": host_info()},
        "roofline": {"bound": "xgmi", "achieved": round(achieved, 2), "peak": link_peak,
                     "unit": "GB/s", "frac": round(achieved / link_peak, 4),
                     "frac_of_target_1071_busbw": round(busbw / TARGET_BUSBW_GBS, 4),
                     # traffic = PMC-measured HBM bytes (the N = 1 line); at N > 1 the
                     # bound is the link, whose bytes come from the executed schedule
                     "traffic": None,
                     "egress_bytes": egress,
                     "link_time_bytes": L,
                     # what the node model (pico_amd/model.py) expects for this
                     # transport and chunk; frac_of_model = model / measured
                     "model_ms": nm.get("model_ms"),
                     "frac_of_model": round(nm["model_ms"] / ms, 4) if nm.get("model_ms") else None,
                     "model": nm,
                     "note": "achieved = this rank's xGMI egress bytes (executed schedule) / ms_per_step "
                             "(the median that also gives value); peak = 153 GB/s per link x egress / link_time_bytes (sum over exchange ops "
                             "of the busiest link's bytes): 153 for the literal one-peer-per-step schedule, up "
                             "to 7 x 153 when every step loads all links; frac_of_target_1071_busbw = busbw / "
                             "(7 x 153), the BASELINE target's denominator"},
        "wall_s": round(st["wall_s"], 4),
    }
    if os.environ.get("BINE_FAKE_HOSTS") == "1":
        # ranks sharing ONE GPU (a rehearsal): no xGMI link carries anything,
        # every rank's bytes go through the one HBM -- that is the bound in
        # play; the link figures stay, labelled for a node
        link = out["roofline"]
        hb = nm.get("hbm_bytes")
        ach = hb * world / (ms * 1e-3) / 1e9 if hb else None
        out["roofline"] = {
            "bound": "hbm", "achieved": _r(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": _r(ach / HBM_PEAK_GBS if ach else None), "traffic": None,
            "algorithmic_bytes_per_call": hb * world if hb else None,
            "model_ms": link["model_ms"], "frac_of_model": link["frac_of_model"], "model": nm,
            "link_roofline_if_node": {k: v for k, v in link.items() if k not in ("model", "model_ms", "frac_of_model")},
            "note": "ranks share ONE GPU: achieved = every rank's HBM bytes of one call (pico_amd/model.py "
                    "hbm_bytes, from the executed schedule) / ms_per_step against the one HBM's peak; "
                    "link_roofline_if_node = the xGMI roofline this line would carry on a node"}
    return out

def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--algo", default="bine_bdw_remap")
    ap.add_argument("--elems", type=int, default=C3_ELEMS)
    ap.add_argument("--relay", default="auto",
                    help="transport at N > 1: auto | off (direct) | flat | relay | relay+flat | flatrs | "
                         "flatrs+flat | flatrs+flat+ag | flatrs+flat+a2a | trees")
    ap.add_argument("--chunk-mib", type=int, default=0, help="N > 1: pipelining chunk (0: try 4/8/16/32/64 MiB)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-extras", action="store_true", help="N > 1: skip the C1/C4/C5 side measurements")
    ap.add_argument("--no-graph-trial", action="store_true", help="N > 1: do not trial HIP-graph replay")
    ap.add_argument("--cpu-budget", type=float, default=5.0)
    args = ap.parse_args()
    if args.gpus > 1 or int(os.environ.get("WORLD_SIZE", "1")) > 1:
        res = bench_allreduce(args.steps, args.warmup, args.elems, args.algo, args.relay, not args.no_extras,
                              args.chunk_mib, not args.no_graph_trial)
        if res is not None:
            print(json.dumps(res), flush=True)
        return
    res = bench_n1(args.steps, args.warmup, not args.no_cpu_baseline, args.cpu_budget)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
