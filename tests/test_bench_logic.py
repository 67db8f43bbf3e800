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


def test_dm_wgs_mode_suffix():
    assert bench.dm_wgs("flatrs+flat") is None and bench.dm_wgs("trees") is None
    assert bench.dm_wgs("flatrs+flat+dm") == 0 and bench.dm_wgs("direct+dm") == 0
    assert bench.dm_wgs("flatrs+flat+dm64") == 64 and bench.dm_wgs("relay+flat+dm16") == 16
