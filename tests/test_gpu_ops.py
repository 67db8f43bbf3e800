"""GPU parity of the logical, bitwise and location MPI_Ops (MPI_LAND / LOR / LXOR /
BAND / BOR / BXOR, MAXLOC / MINLOC on the pair types) -- the predefined operators beyond pico_core's MPI_SUM that
libbine's callers may pass (every reduce-family entry point forwards its
MPI_Op to MPI_Reduce_local, e.g. libbine_allreduce.c:888).

Semantics are MPICH 3.3.2's (logical ops: C truthiness on every type, floats
included, result 0 / 1; bitwise ops: integer types only), pinned by golden
vectors of the real reference on sparsified inputs (tools/make_golden.py
ops_jobs; those cases also run through tests/test_gpu.py's golden test).
Here: the kernels directly (reduce_local, reduce_tree, reduce_batch) on every
dtype with zeros / -0.0 / NaN / denormals, and whole collectives in every
transport setting, bit-exact vs the oracle.
"""
import numpy as np
import pytest

from oracle import oracle as O
from test_gpu import ALL_DT, _host_tree, comms, from_dev, run_loopback, sha, to_dev

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
import pico_amd  # noqa: E402

LOGIC = ["land", "lor", "lxor"]
BITS = ["band", "bor", "bxor"]


def sparse(dtype, n, seed, rank=0):
    """pico_core's generator, sparsified (zeros, -0.0, NaN) as in the goldens;
    floats also get denormals and infinities"""
    x = O.sparsify(O.fill(dtype, n, seed), dtype, rank)
    if dtype in ("float", "double"):
        j = np.arange(n)
        x[j % 13 == 4] = np.finfo(x.dtype).tiny / 4
        x[j % 17 == 6] = -np.inf
    return x


def _valid(dtype, op):
    return not (op in BITS and dtype in ("float", "double"))


def _every_algorithm(P, mode, cases, make):
    """every allreduce and reduce_scatter algorithm on loopback ranks for each
    (op, dtype) in `cases`, literal schedule or flat phases, bit-exact vs the
    oracle (statuses compared where the reference errs); make(dt, n, seed, r)
    builds rank r's input.  Returns the mismatches."""
    flat = mode == "flat"
    for c in comms(P):
        c.set_flat_ag(flat)
        c.set_flat_rs(flat)
    bad = []
    try:
        for op, dt in cases:
            n = 1003
            sb = [make(dt, n, 1234 + r, r) for r in range(P)]
            rc = [n // P + (1 if i == 0 else 0) for i in range(P)]
            sbr = [make(dt, sum(rc), 77 + r, r) for r in range(P)]
            for coll, algos in (("allreduce", AR_ALGOS), ("reduce_scatter", RS_ALGOS)):
                for algo in algos:
                    if coll == "allreduce":
                        want, rets = O.allreduce(algo, sb, dt, op)
                        outs, st = run_loopback(coll, algo, sb, dt, op)
                    else:
                        # permute_remap needs equal blocks (DESIGN.md deviations)
                        r_ = rc if algo != "bine_permute_remap" else [n // P] * P
                        s_ = [x[: sum(r_)] for x in sbr]
                        want, rets = O.reduce_scatter(algo, s_, r_, dt, op)
                        outs, st = run_loopback(coll, algo, s_, dt, op, rcounts=r_)
                    if any(rets) or any(st):
                        if [int(x != 0) for x in st] != [int(x != 0) for x in rets]:
                            bad.append((coll, algo, op, dt, st, rets))
                    elif any(sha(o) != sha(w) for o, w in zip(outs, want)):
                        bad.append((coll, algo, op, dt))
    finally:
        for c in comms(P):
            c.set_flat_ag(False)
            c.set_flat_rs(False)
    return bad


def _tree_and_batch(dtype, ops, make):
    """bine_reduce_tree (2 / 8 / 16 leaves, vector body and a 3-element
    scalar case) and bine_reduce_batch (three windows) vs the oracle"""
    esz = np.dtype(O.NP_DTYPES[dtype]).itemsize
    for op in ops:
        for nl in (2, 8, 16):
            for n in (4099, 3):
                host = [make(dtype, n, 300 + j, j) for j in range(nl)]
                want = _host_tree(host, dtype, op)
                leaves = [to_dev(h, pad=16) for h in host]
                out = torch.zeros(n * esz + 64, dtype=torch.uint8, device="cuda:0")
                assert pico_amd.reduce_tree(leaves, out, n, dtype, op) == 0
                torch.cuda.synchronize()
                assert sha(from_dev(out, dtype, n)) == sha(want), (op, nl, n)
        counts = [5003, 16, 1]
        ins = [make(dtype, c, 40 + k, 0) for k, c in enumerate(counts)]
        ios = [make(dtype, c, 50 + k, 2) for k, c in enumerate(counts)]
        tin, tio = [to_dev(x, pad=16) for x in ins], [to_dev(x, pad=16) for x in ios]
        assert pico_amd.reduce_batch(tin, tio, counts, dtype, op) == 0
        torch.cuda.synchronize()
        for k, c in enumerate(counts):
            exp = ios[k].copy()
            O.reduce_local(ins[k], exp, dtype, op)
            assert sha(from_dev(tio[k], dtype, c)) == sha(exp), (op, k)


def _sparse_pico(dt, n, seed, r):
    return O.sparsify(O.fill(dt, n, seed), dt, r)


@pytest.fixture(scope="module")
def dev():
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    return torch.device("cuda:0")


@pytest.mark.parametrize("dtype", ALL_DT)
@pytest.mark.parametrize("op", LOGIC + BITS)
def test_reduce_local_logic_bits(dev, dtype, op):
    """vector body, head / tail elements and operands not co-aligned mod 16 B"""
    esz = np.dtype(O.NP_DTYPES[dtype]).itemsize
    if not _valid(dtype, op):
        a = to_dev(O.fill(dtype, 64, 1))
        with pytest.raises(pico_amd.BineError):
            pico_amd.reduce_local(a, a.data_ptr(), 64, dtype, op)
        return
    for n in (1, 3, 17, 1000, 100003):
        for shift_a, shift_b in ((0, 0), (1, 1), (1, 0)):
            a = sparse(dtype, n, 11 + n)
            b = sparse(dtype, n, 97 + n, rank=1)
            ta = to_dev(np.concatenate([np.zeros(shift_a, a.dtype), a]))
            tb = to_dev(np.concatenate([np.zeros(shift_b, b.dtype), b]))
            pico_amd.reduce_local(ta.data_ptr() + shift_a * esz, tb.data_ptr() + shift_b * esz, n, dtype, op)
            torch.cuda.synchronize()
            exp = b.copy()
            O.reduce_local(a, exp, dtype, op)
            assert from_dev(tb, dtype, n, shift_b * esz).tobytes() == exp.tobytes(), (n, shift_a, shift_b)


@pytest.mark.parametrize("dtype", ["int8", "uint16", "int32", "int64", "float", "double"])
def test_reduce_tree_and_batch_logic_bits(dev, dtype):
    """the flat reduce-scatter's fused tree kernel and the multi-tree batch
    kernel under the new ops (bitwise ops run byte-wise on integer types)"""
    if dtype in ("float", "double"):
        out = torch.zeros(64, dtype=torch.uint8, device="cuda:0")
        for op in BITS:
            assert pico_amd.reduce_tree([out, out], out, 4, dtype, op) != 0
    _tree_and_batch(dtype, [op for op in LOGIC + BITS if _valid(dtype, op)],
                    lambda dt, n, seed, r: sparse(dt, n, seed, rank=r))


AR_ALGOS = ["bine_bdw_remap", "bine_bdw_static", "bine_bdw_remap_segmented", "bine_lat",
            "bine_block_by_block_any_even", "ring", "rabenseifner", "recursivedoubling"]
RS_ALGOS = ["bine_permute_remap", "bine_send_remap", "bine_static", "bine_block_by_block",
            "bine_block_by_block_any_even", "recursivehalving", "recursive_distance_doubling", "ring", "butterfly"]


@pytest.mark.parametrize("mode", ["literal", "flat"])
@pytest.mark.parametrize("P", [4, 8])
def test_collectives_logic_bits_every_algorithm(dev, P, mode):
    """every reduce-family algorithm under LAND / LXOR (int8, float, double,
    uint8, sparse inputs) and BOR / BXOR (int16, int64, int8), literal
    schedule and with the flat phases (fused tree kernel) -- bit-exact vs the
    oracle"""
    cases = [("land", "int8"), ("land", "float"), ("lxor", "double"), ("lxor", "uint8"), ("bor", "int16"),
             ("bxor", "int64"), ("bxor", "int8")]
    bad = _every_algorithm(P, mode, cases, lambda dt, n, seed, r: sparse(dt, n, seed, rank=r))
    assert not bad, bad[:8]


def test_collective_bitwise_on_float_is_refused(dev):
    """MPICH has no bitwise op on floating types (MPI_ERR_OP): the collective
    returns BINE_ERR_ARG on every rank before any exchange"""
    P = 4
    sb = [O.fill("float", 64, r) for r in range(P)]
    _, st = run_loopback("allreduce", "bine_bdw_remap", sb, "float", "band")
    assert st == [1] * P


# ---- MAXLOC / MINLOC on MPI's (value, index) pair types ----------------------------

PAIRS = ["float_int", "double_int", "long_int", "2int", "short_int"]


@pytest.mark.parametrize("dtype", PAIRS)
@pytest.mark.parametrize("op", ["maxloc", "minloc"])
def test_reduce_local_loc_pairs(dev, dtype, op):
    """MPICH's opmaxloc.c / opminloc.c field by field (ties keep the smaller
    index; NaN values never replace nor get replaced); compared on the defined
    bytes (padding is not part of MPI's type map)"""
    esz = np.dtype(O.NP_DTYPES[dtype]).itemsize
    for n in (1, 3, 17, 1000, 100003):
        for shift in (0, 1):
            a = O.sparsify(O.fill(dtype, n, 11 + n), dtype, 0)
            b = O.sparsify(O.fill(dtype, n, 97 + n), dtype, 1)
            # (np.concatenate would promote the padded struct dtypes to packed ones)
            ha, hb = np.zeros(n + shift, a.dtype), np.zeros(n + shift, b.dtype)
            ha[shift:], hb[shift:] = a, b
            ta, tb = to_dev(ha), to_dev(hb)
            pico_amd.reduce_local(ta.data_ptr() + shift * esz, tb.data_ptr() + shift * esz, n, dtype, op)
            torch.cuda.synchronize()
            exp = b.copy()
            O.reduce_local(a, exp, dtype, op)
            assert sha(from_dev(tb, dtype, n, shift * esz)) == sha(exp), (n, shift)


def test_loc_ops_refuse_other_types(dev):
    """MAXLOC / MINLOC only on pair types, pair types only under them (MPICH:
    MPI_ERR_OP)"""
    t = to_dev(O.fill("float", 64, 1))
    with pytest.raises(pico_amd.BineError):
        pico_amd.reduce_local(t, t.data_ptr(), 16, "float", "maxloc")
    p = to_dev(O.fill("float_int", 64, 1))
    for op in ("sum", "max", "land", "band"):
        with pytest.raises(pico_amd.BineError):
            pico_amd.reduce_local(p, p.data_ptr(), 16, "float_int", op)


@pytest.mark.parametrize("dtype", PAIRS)
def test_reduce_tree_and_batch_loc_pairs(dev, dtype):
    _tree_and_batch(dtype, ("maxloc", "minloc"), _sparse_pico)


@pytest.mark.parametrize("mode", ["literal", "flat"])
@pytest.mark.parametrize("P", [4, 8])
def test_collectives_loc_pairs_every_algorithm(dev, P, mode):
    """every reduce-family algorithm under MAXLOC / MINLOC on 8- and 16-byte
    pair types, literal schedule and flat phases, bit-exact vs the oracle (the
    oracle is pinned by the reference's vectors for the unpadded pair types;
    for the padded ones the reference's copy_buffer copies MPI_Type_size x
    count bytes, libbine_utils.h:176-190, and its outputs are wrong)"""
    cases = [("maxloc", "float_int"), ("minloc", "double_int"), ("maxloc", "short_int"), ("minloc", "2int"),
             ("maxloc", "long_int")]
    bad = _every_algorithm(P, mode, cases, _sparse_pico)
    assert not bad, bad[:8]


# ---- C99 complex types (SUM / PROD) -------------------------------------------------

CPLX = ["c_float_complex", "c_double_complex"]


@pytest.mark.parametrize("dtype", CPLX)
@pytest.mark.parametrize("op", ["sum", "prod"])
def test_reduce_local_complex(dev, dtype, op):
    """MPICH's complex sum / product (a = inout; product re = a.re b.re -
    a.im b.im, im = a.re b.im + a.im b.re, no FMA), zeros and -0.0 parts"""
    esz = np.dtype(O.NP_DTYPES[dtype]).itemsize
    for n in (1, 3, 17, 1000, 100003):
        for shift_a, shift_b in ((0, 0), (1, 1), (1, 0)):
            a = O.sparsify(O.fill(dtype, n, 11 + n), dtype, 0)
            b = O.sparsify(O.fill(dtype, n, 97 + n), dtype, 1)
            ta = to_dev(np.concatenate([np.zeros(shift_a, a.dtype), a]))
            tb = to_dev(np.concatenate([np.zeros(shift_b, b.dtype), b]))
            pico_amd.reduce_local(ta.data_ptr() + shift_a * esz, tb.data_ptr() + shift_b * esz, n, dtype, op)
            torch.cuda.synchronize()
            exp = b.copy()
            O.reduce_local(a, exp, dtype, op)
            assert from_dev(tb, dtype, n, shift_b * esz).tobytes() == exp.tobytes(), (n, shift_a, shift_b)
    with pytest.raises(pico_amd.BineError):
        pico_amd.reduce_local(ta, tb.data_ptr(), 4, dtype, "max")


@pytest.mark.parametrize("dtype", CPLX)
def test_reduce_tree_and_batch_complex(dev, dtype):
    _tree_and_batch(dtype, ("sum", "prod"), _sparse_pico)


@pytest.mark.parametrize("mode", ["literal", "flat"])
@pytest.mark.parametrize("P", [4, 8])
def test_collectives_complex_every_algorithm(dev, P, mode):
    """every reduce-family algorithm under complex SUM / PROD, literal schedule
    and flat phases, bit-exact vs the oracle (pinned by the reference's
    vectors on both complex types)"""
    cases = [("sum", "c_float_complex"), ("prod", "c_double_complex"), ("prod", "c_float_complex")]
    bad = _every_algorithm(P, mode, cases, _sparse_pico)
    assert not bad, bad[:8]