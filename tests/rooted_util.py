"""What the product must do for gather_bine / scatter_bine / alltoall_bine
(libbine_gather.c:16, libbine_scatter.c:14, libbine_alltoall.c:14) -- test
infrastructure shared by the CPU and GPU tests.

The product runs the reference's literal block schedule where the reference
delivers the collective, and refuses the call elsewhere (BINE_ERR_ROOT at a
power-of-two P, BINE_ERR_SIZE otherwise): the oracle's message-level replay
(oracle.gather / scatter / alltoall, pinned by tests/golden) says which.
One deviation: scatter at P = 1 is the copy of the root's block (the
reference shifts by -1 there and crashes, libbine_scatter.c:57)."""
import numpy as np

from oracle import oracle as O

ROOTED = ("gather", "scatter", "alltoall")
ERR_ROOT, ERR_SIZE = 8, 2   # bine_status_t


def intended(coll, sbufs, root, P, n):
    """the collective itself: per-rank outputs (gather: the root's only)"""
    dt = np.asarray(sbufs[root if coll == "scatter" else 0]).dtype   # (np.concatenate drops pair types' padding)

    def cat(parts):
        out = np.zeros(P * n, dt)
        for k, x in enumerate(parts):
            out[k * n:(k + 1) * n] = x
        return out
    if coll == "gather":
        return [cat([np.asarray(s)[:n] for s in sbufs]) if r == root else None for r in range(P)]
    if coll == "scatter":
        return [np.asarray(sbufs[root])[r * n:(r + 1) * n] for r in range(P)]
    return [cat([np.asarray(sbufs[s])[r * n:(r + 1) * n] for s in range(P)]) for r in range(P)]


def replay(coll, sbufs, dt, root, P):
    """the oracle's replay of the reference: (per-rank outputs, rets)"""
    if coll == "gather":
        o, rets = O.gather(sbufs, dt, root)
        return [o if r == root else None for r in range(P)], rets
    if coll == "scatter":
        return O.scatter(np.asarray(sbufs[root]), P, dt, root)
    return O.alltoall(sbufs, dt)


def expect(coll, sbufs, dt, root, P, n):
    """(per-rank outputs or None, bine status) the device path must give"""
    want = intended(coll, sbufs, root, P, n)
    if coll == "scatter" and P == 1:
        return want, 0
    got, rets = replay(coll, sbufs, dt, root, P)
    ok = not isinstance(rets[0], str) and all(
        (w is None) or (g is not None and O.canonical(np.asarray(g)) == O.canonical(np.asarray(w)))
        for g, w in zip(got, want))
    if ok:
        return want, 0
    return None, ERR_ROOT if (P & (P - 1)) == 0 and coll != "alltoall" else ERR_SIZE


def inputs(coll, dt, n, P, seed_base=1234):
    """every rank's send buffer: gather n elements, scatter / alltoall P * n"""
    return O.inputs(dt, n if coll == "gather" else n * P, P, seed_base)


def defined(coll, P, root, n):
    """per rank: a boolean mask of the output elements whose value the
    reference defines -- False where they come from one of its uninitialised
    malloc'd temporaries (the (P, root) pairs at which it returns a wrong
    result), found by replaying the schedule on element tags"""
    tot = n if coll == "gather" else n * P
    sb = [np.array([(r, i) for i in range(tot)] + [None], dtype=object)[:tot] for r in range(P)]
    if coll == "gather":
        out = np.zeros(P * n, object)
        O._run_rooted(P, O._gather_progs(P, n, root, sb, out))
        outs = [out if r == root else np.zeros(0, object) for r in range(P)]
    elif coll == "scatter":
        outs = [np.zeros(n, object) for _ in range(P)]
        O._run_rooted(P, O._scatter_progs(P, n, root, sb[root], outs))
    else:
        outs = [np.zeros(P * n, object) for _ in range(P)]
        O._run_rooted(P, O._alltoall_progs(P, n, sb, outs))
    return [np.array([x is not None for x in o], bool) for o in outs]
