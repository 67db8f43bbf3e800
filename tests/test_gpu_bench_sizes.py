"""GPU parity at the exact shapes bench.py times.

* C3 at P = 1: allreduce_bine_bdw_remap, 256 MiB fp32, through a size-1 RCCL
  communicator -- the reference copies sbuf to rbuf (libbine_allreduce.c:
  849-852); the output's digest must equal the oracle's, which itself equals
  the REAL reference's output digest (profiles/r2_c3_digests_vs_reference.txt).
* C2: the single-launch MPI_Reduce_local kernel on exactly 16,777,216 fp32
  elements (4,096 workgroups), digest vs the oracle's MPICH-semantics result.
* The flat reduce-scatter's tree kernel at its C3 chunk shape, 8 leaves x
  4,194,304 fp32 elements, vs the oracle's pairwise MPI_Reduce_local tree.
* k_copy (copy_buffer): every head / tail / alignment case, byte-exact.
Tolerance: 0 ulp (bit-exact) throughout.
"""
import json
import os

import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
import pico_amd  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
with open(os.path.join(ROOT, "tests", "golden", "bench_digests.json")) as _f:
    GOLD = json.load(_f)["digests"]

C2_N, C3_N = 16_777_216, 67_108_864
TREE_L, TREE_N = 8, 4_194_304


@pytest.fixture(scope="module")
def dev():
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    return torch.device("cuda:0")


def test_c2_reduce_local_full_size_bit_exact(dev):
    a = torch.empty(C2_N, dtype=torch.float32, device=dev)
    b = torch.empty(C2_N, dtype=torch.float32, device=dev)
    pico_amd.fill_pico(a, C2_N, "float", 1234)
    pico_amd.fill_pico(b, C2_N, "float", 1235)
    pico_amd.reduce_local(a, b, C2_N, "float", "sum")
    got = pico_amd.checksum(b, C2_N, "float")
    ha, hb = O.fill("float", C2_N, 1234), O.fill("float", C2_N, 1235)
    O.reduce_local(ha, hb, "float")
    assert got == O.digest(hb) == GOLD[f"C2/reduce_local/sum/float/N{C2_N}"][0]
    # and element for element (64 MiB host copy)
    assert np.array_equal(b.cpu().numpy().view(np.uint32), hb.view(np.uint32))


def test_c3_chunk_reduce_tree_full_shape_bit_exact(dev):
    leaves = [torch.empty(TREE_N, dtype=torch.float32, device=dev) for _ in range(TREE_L)]
    for j, t in enumerate(leaves):
        pico_amd.fill_pico(t, TREE_N, "float", 5000 + j)
    out = torch.empty(TREE_N, dtype=torch.float32, device=dev)
    assert pico_amd.reduce_tree(leaves, out, TREE_N, "float", "sum") == 0
    torch.cuda.synchronize()
    want = O.reduce_tree([O.fill("float", TREE_N, 5000 + j) for j in range(TREE_L)], "float")
    assert np.array_equal(out.cpu().numpy().view(np.uint32), want.view(np.uint32))
    assert O.digest(want) == GOLD[f"tree/reduce_tree/sum/float/N{TREE_N}/L{TREE_L}"][0]


def test_c3_p1_allreduce_size1_rccl_comm(dev):
    comm = pico_amd.Comm.rccl(0, 1, pico_amd.Comm.unique_id(), 0)
    try:
        s = torch.empty(C3_N, dtype=torch.float32, device=dev)
        r = torch.zeros(C3_N, dtype=torch.float32, device=dev)
        pico_amd.fill_pico(s, C3_N, "float", 1234)
        for _ in range(2):   # plan cache reuse
            r.zero_()
            pico_amd.allreduce("bine_bdw_remap", s, r, C3_N, "float", "sum", comm)
            torch.cuda.synchronize()
            comm.synchronize()
            assert pico_amd.checksum(r, C3_N, "float") == GOLD[f"C3/allreduce/bine_bdw_remap/float/N{C3_N}/P1"][0]
        assert torch.equal(r, s)
    finally:
        comm.destroy()


@pytest.mark.parametrize("nbytes", [0, 1, 15, 16, 17, 255, 4096, 4099, 1 << 20, (1 << 20) + 7, 33_554_435])
@pytest.mark.parametrize("off", [0, 1, 8, 13])
def test_copy_kernel_byte_exact(dev, nbytes, off):
    src = torch.randint(0, 256, (nbytes + 64,), dtype=torch.uint8, device=dev)
    dst = torch.zeros(nbytes + 64, dtype=torch.uint8, device=dev)
    pico_amd.copy(dst[off:], src[off:], nbytes)
    torch.cuda.synchronize()
    assert torch.equal(dst[off:off + nbytes], src[off:off + nbytes])
    assert int(dst[:off].sum()) == 0 and int(dst[off + nbytes:].sum()) == 0


def test_copy_kernel_not_coaligned(dev):
    """src / dst not co-aligned mod 16 B: the runtime's device copy"""
    src = torch.randint(0, 256, (100_003,), dtype=torch.uint8, device=dev)
    dst = torch.zeros(100_010, dtype=torch.uint8, device=dev)
    pico_amd.copy(dst[3:], src[0:], 100_003)
    torch.cuda.synchronize()
    assert torch.equal(dst[3:100_006], src)


def test_copy_kernel_c3_size(dev):
    n = C3_N
    s = torch.empty(n, dtype=torch.float32, device=dev)
    pico_amd.fill_pico(s, n, "float", 1234)
    d = torch.empty(n, dtype=torch.float32, device=dev)
    pico_amd.copy(d, s, 4 * n)
    torch.cuda.synchronize()
    assert pico_amd.checksum(d, n, "float") == GOLD[f"C3/allreduce/bine_bdw_remap/float/N{C3_N}/P1"][0]


def test_graph_mode_size1_comm(dev):
    """bine_comm_set_graphs on an RCCL communicator: first call eager +
    captured, later calls replayed; the NULL stream runs eagerly"""
    comm = pico_amd.Comm.rccl(0, 1, pico_amd.Comm.unique_id(), 0)
    try:
        comm.set_graphs(True)
        n = 1 << 20
        s = torch.empty(n, dtype=torch.float32, device=dev)
        pico_amd.fill_pico(s, n, "float", 99)
        r = torch.zeros(n, dtype=torch.float32, device=dev)
        side = torch.cuda.Stream()
        torch.cuda.synchronize()
        for i in range(3):
            with torch.cuda.stream(side):
                r.fill_(float("nan"))
                pico_amd.allreduce("bine_bdw_remap", s, r, n, "float", "sum", comm)
            torch.cuda.synchronize()
            assert torch.equal(r, s), i
        # one rank, no RCCL calls: captured on every runtime (executor.cpp
        # rccl_free; the suite's process runs with 2 HW queues, conftest.py)
        assert comm.graphs_cached() == 1
        r.zero_()
        pico_amd.allreduce("bine_bdw_remap", s, r, n, "float", "sum", comm, stream=0)   # NULL stream: eager
        torch.cuda.synchronize()
        assert torch.equal(r, s)
        comm.set_graphs(False)
        assert comm.graphs_cached() == 0
    finally:
        comm.destroy()


# ---- C1 at its own shape (BASELINE configs[0]) --------------------------------------

C1_N, C1_P = 262_144, 4


@pytest.mark.parametrize("mode", ["direct", "flat", "flatrs+flat", "relay"])
@pytest.mark.parametrize("algo", ["bine_bdw_remap", "bine_lat"])
def test_c1_allreduce_own_shape_vs_committed_digests(dev, algo, mode):
    """C1 itself: fp32 SUM allreduce, 262,144 elements (1 MiB) per rank, P = 4,
    pico_core's inputs (seed 1234 + rank, generated on the device) -- the
    reference's own CPU configuration (pico_core bine_bdw_remap_over,
    libbine_allreduce.c:820-923; bine_lat, :321-439).  Four loopback ranks on
    one MI355X through the same planner and executor as RCCL, literal
    schedule, flat allgather, flat reduce-scatter + flat allgather (the
    one-shot form for bine_lat) and relay; every rank's output digest must
    equal the committed oracle digest (tools/make_bench_digests.py) --
    bine_lat's result differs per rank, as in the reference.  0 ulp."""
    cs = pico_amd.Comm.loopback(C1_P, 0)
    try:
        for c in cs:
            c.set_relay(256 << 10 if mode == "relay" else 0)
            c.set_flat_ag("flat" in mode)
            c.set_flat_rs("flatrs" in mode)
        sb = [torch.empty(C1_N, dtype=torch.float32, device=dev) for _ in range(C1_P)]
        for r, b in enumerate(sb):
            pico_amd.fill_pico(b, C1_N, "float", 1234 + r)
        rb = [torch.full((C1_N,), float("nan"), dtype=torch.float32, device=dev) for _ in range(C1_P)]
        torch.cuda.synchronize()
        for _ in range(3):   # repeated calls reuse the cached plan and workspace
            rc, st = pico_amd.loopback_allreduce(cs, algo, sb, rb, C1_N, "float")
            assert rc == 0 and not any(st), st
        got = [pico_amd.checksum(b, C1_N, "float") for b in rb]
        want = [int(x) for x in GOLD[f"C1/allreduce/{algo}/float/N{C1_N}/P{C1_P}"]]
        assert got == want
    finally:
        for c in cs:
            c.destroy()
