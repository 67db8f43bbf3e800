"""GPU parity at BASELINE.json's full sizes.

Eight virtual ranks on one MI355X (loopback transport, the same planner and
executor as RCCL), inputs generated on the device by k_fill_pico (bit-identical
to pico_core's host generator, tests/test_gpu.py), default 16 MiB pipelining
chunks -- i.e. the exact schedules bench.py times.

* C3 fp32 allreduce 256 MiB/rank: every rank's output digest equals the
  oracle's (the CPU restatement pinned by the reference's vectors) at full
  size, committed in tests/golden/bench_digests.json -- bit-exact, tolerance
  0 ulp; direct, relay and multi-tree transports (trees: vs the relabelled
  oracle).
* C5 int64 allreduce 256 MiB/rank: exact vs the element-wise wrapped int64 sum
  (integer SUM is associative, so any correct schedule gives these bits); fp64
  vs the oracle's digests.
* C4 fp32 reduce_scatter 1 GiB/rank on pico_core's own inputs (seed 1234 +
  rank): every rank's output digest equals the committed oracle digest
  (tests/golden/bench_digests.json), i.e. the reference's association order
  at full size, 0 ulp; direct and flat reduce-scatter (the fused tree
  kernel).  Beside it, integer-valued fp32 inputs (sums of eight values <
  2^24 are exact in any association order) checked element for element
  against a device-side sum, for every transport incl. multi-tree mode.
"""
import json
import os

import numpy as np
import pytest

import _sub

from oracle import oracle as O

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
import pico_amd  # noqa: E402

P = 8
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
with open(os.path.join(ROOT, "tests", "golden", "bench_digests.json")) as _f:
    GOLD = json.load(_f)["digests"]
C3_N = 67_108_864
C4_N = 268_435_456
C5_N = 33_554_432


def _mix64(x):
    x = (x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    x = (x ^ (x >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return x ^ (x >> np.uint64(31))


def host_checksum(a: np.ndarray) -> int:
    """k_checksum's digest on the host, computed in slabs to bound memory"""
    bits_t = {1: np.uint8, 2: np.uint16, 4: np.uint32, 8: np.uint64}[a.dtype.itemsize]
    raw = a.view(bits_t)
    tot = np.uint64(0)
    slab = 1 << 22
    with np.errstate(over="ignore"):
        for s in range(0, a.size, slab):
            bits = raw[s:s + slab].astype(np.uint64)
            idx = np.arange(s, s + bits.size, dtype=np.uint64) * np.uint64(0x9E3779B97F4A7C15)
            tot = tot + _mix64(bits + idx).sum(dtype=np.uint64)
    return int(tot)


@pytest.fixture(scope="module")
def dev():
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    return torch.device("cuda:0")


@pytest.fixture(scope="module")
def comms(dev):
    cs = pico_amd.Comm.loopback(P, 0)
    yield cs
    for c in cs:
        c.destroy()
    torch.cuda.empty_cache()


def _mode(cs, mode):
    for c in cs:
        c.set_relay(256 << 10 if "relay" in mode else 0)  # bench.py RELAY_MIN_BYTES
        c.set_trees(mode == "trees")
        c.set_flat_ag("flat" in mode)
        c.set_flat_rs("flatrs" in mode)


def _device_inputs(dtype, tdt, n):
    bufs = [torch.empty(n, dtype=tdt, device="cuda:0") for _ in range(P)]
    for r, b in enumerate(bufs):
        pico_amd.fill_pico(b, n, dtype, 1234 + r)
    torch.cuda.synchronize()
    return bufs


def test_fill_checksum_consistency_fullsize(dev):
    """the device generator + digest agree with the host at the C3 size"""
    t = torch.empty(C3_N, dtype=torch.float32, device="cuda:0")
    pico_amd.fill_pico(t, C3_N, "float", 1234)
    assert pico_amd.checksum(t, C3_N, "float") == host_checksum(O.fill("float", C3_N, 1234))


def _gold(key):
    return [int(x) for x in GOLD[key]]


@pytest.mark.parametrize("mode", ["direct", "relay", "trees", "flat", "relay+flat", "flatrs+flat"])
def test_c3_allreduce_fullsize(dev, comms, mode):
    """C3 at full size in 8 loopback ranks on pico_core's inputs, every rank's
    digest vs the committed oracle digest (tools/make_bench_digests.py: the
    oracle at full size; equal to the real reference's, profiles/
    r2_c3_digests_vs_reference.txt); trees: vs the relabelled schedule's
    digest.  (Round 3 recomputed the oracle on the host here -- the same
    digests at a minute of CPU time per run.)"""
    key = f"C3/allreduce/bine_bdw_remap/float/N{C3_N}/P{P}"
    digests = _gold(key)
    assert len(set(digests)) == 1  # allreduce: every rank holds the same bits
    expect = _gold(key + "/trees") if mode == "trees" else digests
    sb = _device_inputs("float", torch.float32, C3_N)
    rb = [torch.empty(C3_N, dtype=torch.float32, device="cuda:0") for _ in range(P)]
    _mode(comms, mode)
    try:
        rc, st = pico_amd.loopback_allreduce(comms, "bine_bdw_remap", sb, rb, C3_N, "float")
        assert rc == 0 and not any(st), st
        got = [pico_amd.checksum(b, C3_N, "float") for b in rb]
    finally:
        _mode(comms, "direct")
    assert got == expect


@pytest.mark.parametrize("mode", ["direct", "relay", "trees", "flatrs+flat"])
def test_c5_int64_allreduce_fullsize(dev, comms, mode):
    sb = _device_inputs("int64", torch.int64, C5_N)
    want = sb[0].clone()
    for b in sb[1:]:
        want.add_(b)  # two's-complement wrap, same as MPICH's int64 SUM
    rb = [torch.empty(C5_N, dtype=torch.int64, device="cuda:0") for _ in range(P)]
    _mode(comms, mode)
    try:
        rc, st = pico_amd.loopback_allreduce(comms, "bine_bdw_remap", sb, rb, C5_N, "int64")
        assert rc == 0 and not any(st), st
        torch.cuda.synchronize()
        assert all(torch.equal(b, want) for b in rb)
    finally:
        _mode(comms, "direct")


@pytest.mark.parametrize("mode", ["direct", "flatrs+flat"])
def test_c5_double_allreduce_fullsize(dev, comms, mode):
    expect = _gold(f"C5/allreduce/bine_bdw_remap/double/N{C5_N}/P{P}")[0]  # the committed oracle digest
    sb = _device_inputs("double", torch.float64, C5_N)
    rb = [torch.empty(C5_N, dtype=torch.float64, device="cuda:0") for _ in range(P)]
    _mode(comms, mode)
    try:
        rc, st = pico_amd.loopback_allreduce(comms, "bine_bdw_remap", sb, rb, C5_N, "double")
        assert rc == 0 and not any(st), st
        got = [pico_amd.checksum(b, C5_N, "double") for b in rb]
    finally:
        _mode(comms, "direct")
    assert got == [expect] * P


@pytest.mark.parametrize("mode", ["direct", "flatrs", "relay"])
def test_c4_reduce_scatter_fullsize_pico_inputs(dev, comms, mode):
    """C4 exactly as bench.py runs it: reduce_scatter_bine_permute_remap, fp32
    SUM, 268,435,456 elements (1 GiB) per rank at P = 8, pico_core's
    distribution (rand_r / RAND_MAX * 100, seed 1234 + rank,
    pico_core_utils.c:903-916) -- every rank's 128 MiB block digest equals the
    oracle's digest of the reference's association order
    (libbine_reduce_scatter.c:985-1063), committed in
    tests/golden/bench_digests.json.  (pico_core's generator repeats every
    2^27 elements, so blocks r and r + 4 carry equal digests; the element-wise
    test below uses non-repeating inputs.)"""
    per = C4_N // P
    want = [int(x) for x in GOLD[f"C4/reduce_scatter/bine_permute_remap/float/N{C4_N}/P{P}"]]
    sb = _device_inputs("float", torch.float32, C4_N)
    rb = [torch.full((per,), float("nan"), dtype=torch.float32, device="cuda:0") for _ in range(P)]
    torch.cuda.synchronize()
    _mode(comms, mode)
    try:
        rc, st = pico_amd.loopback_reduce_scatter(comms, "bine_permute_remap", sb, rb, [per] * P, "float")
        assert rc == 0 and not any(st), st
        torch.cuda.synchronize()
        got = [pico_amd.checksum(b, per, "float") for b in rb]
    finally:
        _mode(comms, "direct")
        del sb, rb
        torch.cuda.empty_cache()
    assert got == want


@pytest.mark.parametrize("mode", ["direct", "relay", "trees", "flatrs"])
def test_c4_reduce_scatter_fullsize(dev, comms, mode):
    per = C4_N // P
    g = torch.Generator(device="cuda:0")
    g.manual_seed(4)
    sb = [torch.randint(0, 1 << 20, (C4_N,), generator=g, device="cuda:0", dtype=torch.int32).float()
          for _ in range(P)]
    rb = [torch.empty(per, dtype=torch.float32, device="cuda:0") for _ in range(P)]
    # the loopback drivers run on the communicators' own (non-blocking) streams:
    # torch's generator kernels must be finished before they start
    torch.cuda.synchronize()
    _mode(comms, mode)
    try:
        rc, st = pico_amd.loopback_reduce_scatter(comms, "bine_permute_remap", sb, rb, [per] * P, "float")
        assert rc == 0 and not any(st), st
        torch.cuda.synchronize()
    finally:
        _mode(comms, "direct")
    for r in range(P):
        want = sb[0][r * per:(r + 1) * per].clone()
        for b in sb[1:]:
            want.add_(b[r * per:(r + 1) * per])
        assert torch.equal(rb[r], want), r
    del sb, rb
    torch.cuda.empty_cache()


@pytest.mark.parametrize("algo,flat", [("bine_bdw_remap", False), ("bine_bdw_remap", True), ("ring", False)])
def test_allreduce_beyond_int32_element_counts(dev, algo, flat):
    """counts past 2^31 elements (the reference's reduce_scatter takes int
    rcounts; its allreduce takes size_t counts): int8 SUM allreduce of
    2^31 + 4099 elements per rank at P = 2 -- every 32-bit index or grid
    computation in the planner, executor and kernels would show here.
    Integer SUM is associative, so the wrapped element-wise sum is the exact
    result of any schedule; it is computed on the device in int16."""
    n = (1 << 31) + 4099
    cs = pico_amd.Comm.loopback(2, 0)
    try:
        for c in cs:
            c.set_flat_ag(flat)
            c.set_flat_rs(flat)
        sb = [torch.empty(n, dtype=torch.int8, device="cuda:0") for _ in range(2)]
        for r, b in enumerate(sb):
            pico_amd.fill_pico(b, n, "int8", 1234 + r)
        rb = [torch.empty(n, dtype=torch.int8, device="cuda:0") for _ in range(2)]
        torch.cuda.synchronize()
        rc, st = pico_amd.loopback_allreduce(cs, algo, sb, rb, n, "int8")
        assert rc == 0 and not any(st), st
        torch.cuda.synchronize()
        want = torch.empty(n, dtype=torch.int8, device="cuda:0")
        step = 1 << 28
        for s in range(0, n, step):   # (a + b) mod 2^8, in slabs to bound the int16 temporaries
            want[s:s + step] = (sb[0][s:s + step].to(torch.int16) + sb[1][s:s + step].to(torch.int16)).to(torch.int8)
        for r in range(2):
            assert torch.equal(rb[r], want), r
    finally:
        for c in cs:
            c.destroy()
        torch.cuda.empty_cache()


@pytest.mark.parametrize("algo", ["bine_permute_remap", "bine_block_by_block", "recursivehalving"])
def test_reduce_scatter_beyond_int32_total(dev, algo):
    """int rcounts (include/libbine.h REDUCE_SCATTER_ARGS) whose total passes
    2^31 elements: int8 SUM at P = 2, blocks of 2^30 + 5, exact vs the
    wrapped element-wise sum of each block"""
    blk = (1 << 30) + 5
    n = 2 * blk
    cs = pico_amd.Comm.loopback(2, 0)
    try:
        sb = [torch.empty(n, dtype=torch.int8, device="cuda:0") for _ in range(2)]
        for r, b in enumerate(sb):
            pico_amd.fill_pico(b, n, "int8", 4321 + r)
        rb = [torch.empty(blk, dtype=torch.int8, device="cuda:0") for _ in range(2)]
        torch.cuda.synchronize()
        rc, st = pico_amd.loopback_reduce_scatter(cs, algo, sb, rb, [blk, blk], "int8")
        assert rc == 0 and not any(st), st
        torch.cuda.synchronize()
        for r in range(2):
            lo = r * blk
            want = (sb[0][lo:lo + blk].to(torch.int16) + sb[1][lo:lo + blk].to(torch.int16)).to(torch.int8)
            assert torch.equal(rb[r], want), r
            del want
    finally:
        for c in cs:
            c.destroy()
        torch.cuda.empty_cache()


@pytest.mark.timeout(700)
def test_full_size_configs_eight_processes():
    """C3 (fp32 256 MiB/rank), C4 (reduce_scatter 1 GiB/rank) and C5 (fp64,
    int64 256 MiB/rank) at P = 8 in eight real processes -- the transports the
    driver's 8-GPU bench picks from (flat phases and the literal schedule over
    the direct peer-memory transport, the flat phases over RCCL P2P) -- every
    rank's output digest equal to the committed oracle digest of pico_core's
    inputs (tools/fullsize_multirank.py)"""
    import sys
    env = dict(os.environ, PYTHONPATH=ROOT)
    r = _sub.run_kw([sys.executable, "-u", os.path.join(ROOT, "tools", "fullsize_multirank.py"), "8"], env=env,
                       capture_output=True, text=True, timeout=680, ranks=8)
    # every MISMATCH line first (which case, on which rank), then the tail
    bad = [x for x in r.stdout.splitlines() if "MISMATCH" in x]
    tail = "\n".join(bad[:64] + r.stdout.splitlines()[-12:])
    assert r.returncode == 0, tail + "\n" + r.stderr[-1500:]
    assert "RESULT P=8: ok" in r.stdout
