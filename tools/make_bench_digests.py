#!/usr/bin/env python3
"""Golden digests for bench.py's in-run parity checks (TEST INFRASTRUCTURE).

bench.py checks the output of every transport trial and of every timed
configuration against these digests (bine_checksum of the device buffer vs
the value here), so the driver's only multi-GPU run carries its own parity
evidence, as pico_core checks every benchmark run against PMPI_*
(pico_core/pico_core_utils.c:553-610).  The values come from the oracle (the
CPU restatement pinned bit for bit by the reference's golden vectors,
tests/test_oracle.py) on the bench's exact inputs: pico_core's rand_r
distribution with seed 1234 + rank (pico_core_utils.c:902-923), generated on
the device by k_fill_pico (bit-identical, tests/test_gpu.py).

Keys: "<config>/<collective>/<algorithm>/<dtype>/N<count>/P<ranks>[/trees]" ->
list of per-rank digests (reduce_scatter: digest of rank r's block).  "/trees"
= multi-tree mode: the reference schedule on relabelled ranks per slice
(tests/test_trees.py), which differs from the reference in fp rounding only.

usage: python tools/make_bench_digests.py [--quick]   (--quick: C1 / C2 / tree only)
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from oracle import oracle as O  # noqa: E402

OUT = os.path.join(ROOT, "tests", "golden", "bench_digests.json")

C1_N, C2_N, C3_N, C4_N, C5_N = 262_144, 16_777_216, 67_108_864, 268_435_456, 33_554_432
TREE_LEAVES, TREE_N, TREE_SEED = 8, 4_194_304, 5000


def key(cfg, coll, algo, dtype, n, P, trees=False):
    return f"{cfg}/{coll}/{algo}/{dtype}/N{n}/P{P}" + ("/trees" if trees else "")


def small():
    d = {}
    for algo in ("bine_bdw_remap", "bine_lat"):
        for P in (2, 4, 8):
            sb = O.inputs("float", C1_N, P)
            want, rets = O.allreduce(algo, sb, "float")
            assert not any(rets)
            d[key("C1", "allreduce", algo, "float", C1_N, P)] = [O.digest(w) for w in want]
    a, b = O.fill("float", C2_N, 1234), O.fill("float", C2_N, 1235)
    O.reduce_local(a, b, "float")
    d[f"C2/reduce_local/sum/float/N{C2_N}"] = [O.digest(b)]
    leaves = [O.fill("float", TREE_N, TREE_SEED + j) for j in range(TREE_LEAVES)]
    d[f"tree/reduce_tree/sum/float/N{TREE_N}/L{TREE_LEAVES}"] = [O.digest(O.reduce_tree(leaves, "float"))]
    return d


R64_F, R64_D = 16_777_216, 8_388_608   # tools/rccl_large.py: 64 MiB per rank in fp32 / fp64


def rccl_large():
    """tools/rccl_large.py's cases (64 MiB per rank, P = 2, 4, 8): the inputs'
    own digests (so a rank can tell a corrupted input from a wrong result),
    allreduce_bine_bdw_remap fp32 / fp64 (+ multi-tree at P = 4, 8) and
    reduce_scatter_bine_permute_remap fp32"""
    import test_trees as TT
    d = {}
    for dt, n in (("float", R64_F), ("double", R64_D)):
        d[key("L64", "input", "fill_pico", dt, n, 8)] = [O.digest(O.fill(dt, n, 1234 + r)) for r in range(8)]
    for P in (2, 4, 8):
        for dt, n in (("float", R64_F), ("double", R64_D)):
            sb = O.inputs(dt, n, P)
            want, rets = O.allreduce("bine_bdw_remap", sb, dt)
            assert not any(rets)
            d[key("L64", "allreduce", "bine_bdw_remap", dt, n, P)] = [O.digest(w) for w in want]
            if P in (4, 8):
                want = TT.relabelled_oracle("bine_bdw_remap", sb, dt)
                d[key("L64", "allreduce", "bine_bdw_remap", dt, n, P, True)] = [O.digest(w) for w in want]
        sb = O.inputs("float", R64_F, P)
        want, rets = O.reduce_scatter("bine_permute_remap", sb, [R64_F // P] * P, "float")
        assert not any(rets)
        d[key("L64", "reduce_scatter", "bine_permute_remap", "float", R64_F, P)] = [O.digest(w) for w in want]
        print(f"L64 P={P}", flush=True)
    return d


def big():
    import test_trees as TT
    d = {}
    for P in (1, 2, 4, 8):
        t0 = time.time()
        sb = O.inputs("float", C3_N, P)
        want, rets = O.allreduce("bine_bdw_remap", sb, "float")
        assert not any(rets)
        d[key("C3", "allreduce", "bine_bdw_remap", "float", C3_N, P)] = [O.digest(w) for w in want]
        if P in (4, 8):
            want = TT.relabelled_oracle("bine_bdw_remap", sb, "float")
            d[key("C3", "allreduce", "bine_bdw_remap", "float", C3_N, P, True)] = [O.digest(w) for w in want]
        del sb, want
        print(f"C3 P={P} {time.time() - t0:.1f} s", flush=True)
    for dt in ("double", "int64"):
        for P in (2, 4, 8):
            t0 = time.time()
            sb = O.inputs(dt, C5_N, P)
            want, rets = O.allreduce("bine_bdw_remap", sb, dt)
            assert not any(rets)
            d[key("C5", "allreduce", "bine_bdw_remap", dt, C5_N, P)] = [O.digest(w) for w in want]
            if P in (4, 8):
                want = TT.relabelled_oracle("bine_bdw_remap", sb, dt)
                d[key("C5", "allreduce", "bine_bdw_remap", dt, C5_N, P, True)] = [O.digest(w) for w in want]
            del sb, want
            print(f"C5 {dt} P={P} {time.time() - t0:.1f} s", flush=True)
    for P in (2, 4, 8):
        t0 = time.time()
        rc = [C4_N // P] * P
        sb = O.inputs("float", C4_N, P)
        want, rets = O.reduce_scatter("bine_permute_remap", sb, rc, "float")
        assert not any(rets)
        d[key("C4", "reduce_scatter", "bine_permute_remap", "float", C4_N, P)] = [O.digest(w) for w in want]
        del want
        if P in (4, 8):
            want = TT.relabelled_rs_oracle(sb, rc, "float")
            d[key("C4", "reduce_scatter", "bine_permute_remap", "float", C4_N, P, True)] = [O.digest(w) for w in want]
            del want
        del sb
        print(f"C4 P={P} {time.time() - t0:.1f} s", flush=True)
    return d


def main():
    quick = "--quick" in sys.argv
    d = {}
    if os.path.exists(OUT):
        with open(OUT) as f:
            d = json.load(f).get("digests", {})
    d.update(small())
    d.update(rccl_large())
    if not quick:
        d.update(big())
    doc = {"generator": "tools/make_bench_digests.py (oracle/bine_oracle.c, pinned by tests/golden/index.json.gz)",
           "inputs": "pico_core rand_r distribution, seed 1234 + rank (C2: in 1234, inout 1235; tree: leaf j "
                     f"seed {TREE_SEED} + j)",
           "digest": "sum_i mix64(bits(x[i]) + i * 0x9E3779B97F4A7C15) mod 2^64 (bine_checksum)",
           "digests": dict(sorted(d.items()))}
    with open(OUT, "w") as f:
        json.dump(doc, f, indent=1)
    print(f"wrote {len(d)} entries to {OUT}")


if __name__ == "__main__":
    main()
