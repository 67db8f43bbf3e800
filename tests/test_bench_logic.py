"""bench.py's transport choice (host logic only): the fastest transport, but a
bit-exact one over multi-tree mode unless trees wins by more than 3 %."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def test_prefer_bit_exact_transport():
    assert bench._prefer_exact({"direct": 10.0, "trees": 5.0, "flatrs+flat": 5.1}) == "flatrs+flat"
    assert bench._prefer_exact({"direct": 10.0, "trees": 5.0, "flatrs+flat": 6.0}) == "trees"
    assert bench._prefer_exact({"direct": 3.0, "trees": 5.0}) == "direct"
    assert bench._prefer_exact({"trees": 5.0}) == "trees"
    assert bench._prefer_exact({"relay": 4.0, "flat": 4.5}) == "relay"


def test_pick_headline():
    base, best = ("direct", 16, False), ("flatrs+flat", 32, True)
    fast, slow = {"median_ms": 1.0}, {"median_ms": 2.0}
    assert bench.pick_headline(base, (slow, True, 1), best, None) == (base, (slow, True, 1))
    assert bench.pick_headline(base, (slow, True, 1), best, (fast, True, 2))[0] == best
    assert bench.pick_headline(base, (fast, True, 1), best, (slow, True, 2))[0] == base
    # a failed check never wins over a passing (or unchecked) run, however fast
    assert bench.pick_headline(base, (slow, True, 1), best, (fast, False, 2))[0] == base
    assert bench.pick_headline(base, (fast, False), best, (slow, None, 2))[0] == best
    assert bench.pick_headline(base, (fast, False), best, (slow, False, 2))[0] == base


def test_runner_up_after_a_failed_pick():
    inf = float("inf")
    base, a, b, c = ("direct", 16, False), ("x+dmt", 32, False), ("x+dm", 32, False), ("x+dmt256", 32, False)
    trials = {base: 300.0, a: 2.1, b: 19.0, c: inf}
    assert bench.runner_up(trials, a, base) == b
    assert bench.runner_up({base: 300.0, a: 2.1, c: inf}, a, base) is None


def test_dm_wgs_mode_suffix():
    assert bench.dm_wgs("flatrs+flat") is None and bench.dm_wgs("trees") is None
    assert bench.dm_wgs("flatrs+flat+dm") == 0 and bench.dm_wgs("direct+dm") == 0
    assert bench.dm_wgs("flatrs+flat+dm64") == 64 and bench.dm_wgs("relay+flat+dm16") == 16


def test_step_profile_counts_trees_inside_exchanges_as_no_local_time():
    # bine_comm_profile: a fused tree evaluated inside an exchange launch
    # reports nprims 0 / bytes 0 (include/bine_amd.h); it is neither local
    # busy time nor an HBM rate
    class Comm:
        def set_profile(self, on):
            pass

        def synchronize(self):
            pass

        def profile(self):
            return [{"xchg": 1, "nprims": 14, "bytes": 1 << 20, "start_ms": 0.0, "ms": 0.5},
                    {"xchg": 0, "nprims": 0, "bytes": 0, "start_ms": 0.1, "ms": 0.006},
                    {"xchg": 0, "nprims": 1, "bytes": 3 << 20, "start_ms": 0.6, "ms": 0.2}]

    class Torch:
        class cuda:
            @staticmethod
            def synchronize():
                pass

    p = bench.step_profile(Torch, Comm(), lambda: None)
    assert p["local_busy_ms"] == 0.2 and p["ops"] == 3
    assert p["local"][0]["inside_exchange"] and p["local"][0]["hbm_GBs"] is None
    assert "inside_exchange" not in p["local"][1] and p["local"][1]["hbm_GBs"] > 0
