"""The golden digests bench.py checks its own outputs against
(tests/golden/bench_digests.json, tools/make_bench_digests.py), and the bench's
host-side logic.  CPU only.

The small entries (C1 at P = 2, 4, 8; C2; the tree kernel's shape) are
recomputed here with the oracle; C3 at P = 1 is the digest of pico_core's
seed-1234 input (the reference's P = 1 allreduce copies it).  The full-size
C3 entries at P = 1, 2, 4, 8 were also checked against the REAL reference's
output digests (oracle/_ref/ref_bench; profiles/r2_c3_digests_vs_reference.txt),
and bench.py re-checks them in every N = 1 run through the cpu_baseline leg.
"""
import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from oracle import oracle as O  # noqa: E402

with open(os.path.join(ROOT, "tests", "golden", "bench_digests.json")) as f:
    GOLD = json.load(f)["digests"]


def test_every_bench_key_has_a_digest():
    for P in (2, 4, 8):
        for algo in ("bine_bdw_remap", "bine_lat"):
            assert len(GOLD[bench.gkey("C1", "allreduce", algo, "float", bench.C1_ELEMS, P)]) == P
        assert len(GOLD[bench.gkey("C3", "allreduce", "bine_bdw_remap", "float", bench.C3_ELEMS, P)]) == P
        assert len(GOLD[bench.gkey("C4", "reduce_scatter", "bine_permute_remap", "float", bench.C4_ELEMS, P)]) == P
        for dt in ("double", "int64"):
            assert len(GOLD[bench.gkey("C5", "allreduce", "bine_bdw_remap", dt, bench.C5_ELEMS, P)]) == P
    for P in (4, 8):   # multi-tree mode: the relabelled schedule's digests
        assert len(GOLD[bench.gkey("C3", "allreduce", "bine_bdw_remap", "float", bench.C3_ELEMS, P, True)]) == P
        assert len(GOLD[bench.gkey("C4", "reduce_scatter", "bine_permute_remap", "float", bench.C4_ELEMS, P,
                                   True)]) == P
    assert bench.golden(bench.gkey("C3", "allreduce", "bine_bdw_remap", "float", bench.C3_ELEMS, 1)) is not None


@pytest.mark.parametrize("P", [2, 4, 8])
@pytest.mark.parametrize("algo", ["bine_bdw_remap", "bine_lat"])
def test_c1_digests_match_oracle(P, algo):
    want, rets = O.allreduce(algo, O.inputs("float", bench.C1_ELEMS, P), "float")
    assert not any(rets)
    assert [O.digest(w) for w in want] == GOLD[bench.gkey("C1", "allreduce", algo, "float", bench.C1_ELEMS, P)]


def test_c2_and_tree_digests_match_oracle():
    a, b = O.fill("float", bench.C2_ELEMS, 1234), O.fill("float", bench.C2_ELEMS, 1235)
    O.reduce_local(a, b, "float")
    assert O.digest(b) == GOLD[f"C2/reduce_local/sum/float/N{bench.C2_ELEMS}"][0]
    leaves = [O.fill("float", bench.TREE_ELEMS, bench.TREE_SEED + j) for j in range(bench.TREE_LEAVES)]
    tree = O.reduce_tree(leaves, "float")
    assert O.digest(tree) == GOLD[f"tree/reduce_tree/sum/float/N{bench.TREE_ELEMS}/L{bench.TREE_LEAVES}"][0]


def test_c3_p1_digest_is_the_input():
    assert O.digest(O.fill("float", bench.C3_ELEMS, 1234)) == \
        GOLD[bench.gkey("C3", "allreduce", "bine_bdw_remap", "float", bench.C3_ELEMS, 1)][0]


def test_oracle_reduce_tree_is_pairwise_reduce_local():
    """the tree helper = the literal schedule's pairwise MPI_Reduce_local calls,
    incl. the swapped level of block_by_block (libbine_reduce_scatter.c:1143)"""
    import numpy as np
    L = [O.fill("float", 1000, 40 + j) for j in range(4)]
    v0, v1, v2, v3 = (x.copy() for x in L)
    O.reduce_local(v1, v0, "float")
    O.reduce_local(v3, v2, "float")
    O.reduce_local(v2, v0, "float")
    assert np.array_equal(O.reduce_tree(L, "float"), v0)
    # level 1 swapped: v2 (op) v0 with v2 as inout
    v0, v1, v2, v3 = (x.copy() for x in L)
    O.reduce_local(v1, v0, "float")
    O.reduce_local(v3, v2, "float")
    O.reduce_local(v0, v2, "float")
    assert np.array_equal(O.reduce_tree(L, "float", swap=2), v2)


def test_overlap_fraction():
    assert bench.overlap_frac([(0.0, 10.0)], [(2.0, 4.0)]) == 1.0                  # reductions fully hidden
    assert bench.overlap_frac([(0.0, 10.0)], [(10.0, 4.0)]) == 0.0                 # serial
    assert bench.overlap_frac([(0.0, 10.0)], [(8.0, 4.0)]) == 0.5
    assert bench.overlap_frac([(0.0, 5.0), (4.0, 3.0)], [(6.0, 2.0), (9.0, 1.0)]) == 1 / 3   # union of exchanges
    assert bench.overlap_frac([(0.0, 1.0)], []) is None


def test_transport_modes():
    assert bench.transport_modes("auto", 2) == ["direct", "flat", "flatrs+flat", "direct+dm", "flatrs+flat+dm",
                                                "flatrs+flat+dmt"]
    assert "trees" in bench.transport_modes("auto", 8) and "flatrs+flat+ag" in bench.transport_modes("auto", 8)
    assert bench.transport_modes("flatrs+flat+a2a", 8) == ["flatrs+flat+a2a"]
    assert bench.transport_modes("auto", 6) == ["direct", "relay", "direct+dm"]
    assert "relay+flat+dm" in bench.transport_modes("auto", 8)
    assert "flatrs+flat+dmt" in bench.transport_modes("auto", 8)
    assert bench.dm_wgs("flatrs+flat+dmt16") == 16 and bench.dm_tree("flatrs+flat+dmt16") == 1
    assert bench.dm_wgs("flatrs+flat+dm64") == 64 and bench.dm_tree("flatrs+flat+dm64") == 0
    assert bench.dm_wgs("flatrs+flat+dmtx128") == 0 and bench.dm_tree("flatrs+flat+dmtx128") == 128
    assert bench.dm_wgs("flatrs+flat+dmt16x256") == 16 and bench.dm_tree("flatrs+flat+dmt16x256") == 256
    assert bench.dm_wgs("flatrs+flat") is None and bench.dm_tree("direct") == 0
    assert bench.transport_modes("off", 8) == ["direct"]
    assert bench.transport_modes("trees", 2) == ["direct"]


def test_all_ok_without_dist():
    assert bench.all_ok(None, None, True) is True
    assert bench.all_ok(None, None, False) is False
    assert bench.all_ok(None, None, None) is None


def test_arm_deadline_prints_partial_line_and_exits(tmp_path):
    """a side measurement that hangs past the budget: the line measured so far
    is printed, marked cut_by_deadline, and the process ends with the distinct
    status bench.DEADLINE_EXIT (bench.arm_deadline), so a hang never looks
    like a clean run"""
    import subprocess
    import sys
    script = (
        "import sys, time; sys.path.insert(0, %r)\n"
        "import bench\n"
        "out = {'metric': 'm', 'value': 1.0, 'config': {}}\n"
        "def partial():\n"
        "    out['config']['side_measurements_cut_after_s'] = 0.3\n"
        "    return out\n"
        "bench.arm_deadline(0.3, partial, 'side measurements')\n"
        "time.sleep(30)\n"
        "print('not reached')\n" % ROOT)
    r = subprocess.run([sys.executable, "-c", script], capture_output=True, text=True, timeout=60)
    assert r.returncode == bench.DEADLINE_EXIT != 0
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert lines == [{"metric": "m", "value": 1.0, "config": {"side_measurements_cut_after_s": 0.3},
                      "cut_by_deadline": "side measurements"}]
    assert "not reached" not in r.stdout and "exceeded" in r.stderr


def test_arm_deadline_cancelled_is_silent():
    import time
    t = bench.arm_deadline(0.2, lambda: {"x": 1}, "test")
    t.cancel()
    time.sleep(0.4)   # still alive: the timer did not fire


def test_best_of_picks_fastest_verified_rccl_trial():
    inf = float("inf")
    trials = {("direct", 16 << 20, False): 3.0, ("flat", 16 << 20, False): 2.0,
              ("flatrs+flat", 16 << 20, False): 1.0, ("direct+dm", 16 << 20, False): 0.5,
              ("relay", 16 << 20, False): inf}
    verdicts = {("direct", 16 << 20, False): True, ("flat", 16 << 20, False): True,
                ("flatrs+flat", 16 << 20, False): False, ("direct+dm", 16 << 20, False): True,
                ("relay", 16 << 20, False): "error"}
    b = bench._best_of(trials, verdicts, 1 << 28, lambda c: "+dm" not in c[0])
    assert b == {"transport": "flat/16MiB", "ms": 2.0, "algbw_per_rank_GBs": round((1 << 28) / 2e-3 / 1e9, 2)}
    assert bench._best_of(trials, verdicts, 1 << 28, lambda c: False) is None


def test_pmc_traffic_only_for_the_measured_kernel_source(tmp_path, monkeypatch):
    """traffic comes from profiles/latest_pmc.json only while the tree's
    kernels.hip hashes to the source those counters were taken on"""
    pmc = {"kernels_hip_sha256": bench.kernels_source_sha256(),
           "kernels": {"k_copy": {"hbm_bytes_per_launch": 123.0}}}
    (tmp_path / "profiles").mkdir()
    (tmp_path / "pico_amd" / "csrc").mkdir(parents=True)
    with open(os.path.join(ROOT, "pico_amd", "csrc", "kernels.hip"), "rb") as f:
        (tmp_path / "pico_amd" / "csrc" / "kernels.hip").write_bytes(f.read())
    (tmp_path / "profiles" / "latest_pmc.json").write_text(json.dumps(pmc))
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    assert bench._pmc_traffic("k_copy") == 123.0
    (tmp_path / "pico_amd" / "csrc" / "kernels.hip").write_bytes(b"// another build\n")
    assert bench._pmc_traffic("k_copy") is None
