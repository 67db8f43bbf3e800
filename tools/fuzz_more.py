"""The GPU fuzz of tests/test_gpu_fuzz.py over more seeds than the suite runs
(seeds 100 ... 100 + N - 1, 60 random configurations each: collective x
algorithm x P x count x type x operator x transport setting x in place on
loopback ranks, bit-exact vs the oracle or the expected error), then as many
seeds of the bcast and gather / scatter / alltoall sweeps.
usage: python tools/fuzz_more.py N   (prints RESULT <cases> cases <bad> bad)"""
import os, random, sys
ROOT = os.environ.get("GRAFT_REPO_ROOT", "/root/repo")
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
import numpy as np
import torch
np.seterr(all="ignore")
import test_gpu_fuzz as F
import rooted_util as R
from test_gpu import comms, run_loopback, sha
from oracle import oracle as O
bad = []
n = 0
for seed in range(100, 100 + int(sys.argv[1])):
    rng = random.Random(1000 + seed)
    for _ in range(60):
        coll, algo, P, dt, op, nn, o = F._case(rng)
        try:
            want, rets, outs, st = F._run(coll, algo, P, dt, op, nn, o)
        except Exception as e:
            bad.append((seed, coll, algo, P, dt, op, nn, o, "exc", repr(e)[:200])); continue
        n += 1
        if any(rets):
            if list(st) != F.expected_status(rets):
                bad.append((seed, coll, algo, P, dt, op, nn, o, "errors", rets, st))
        elif any(st):
            bad.append((seed, coll, algo, P, dt, op, nn, o, "status", st))
        elif any(sha(x) != sha(w) for x, w in zip(outs, want)):
            bad.append((seed, coll, algo, P, dt, op, nn, o, "data"))
    for PP in (1, 2, 3, 4, 5, 6, 8, 16):
        for c in comms(PP):
            c.set_relay(0); c.set_flat_ag(False); c.set_flat_rs(False); c.set_chunk(0); c.set_trees(False)
    print(f"seed {seed}: {n} cases, {len(bad)} bad", flush=True)
# bcast (every algorithm, any root) and gather / scatter / alltoall, as the
# suite's test_random_bcast_bit_exact / test_random_rooted_bit_exact
nb = 0
for seed in range(100, 100 + int(sys.argv[1])):
    rng = random.Random(5000 + seed)
    for _ in range(20):
        algo = rng.choice(F.COLLS["bcast"])
        P = rng.choice([1, 2, 3, 4, 4, 6, 8, 8, 16])
        dt = rng.choice(list(F.OPS_OF))
        nn = rng.choice([1, 2, 7, 64, 333, 1000, 4097, rng.randint(1, 30000)])
        o = {"relay": rng.choice([0, 0, 64, 4096]), "flat_ag": rng.random() < 0.4, "sparse": rng.random() < 0.5}
        want, rets, outs, st = F._run("bcast", algo, P, dt, "sum", nn, o)
        nb += 1
        if any(rets):
            if list(st) != F.expected_status(rets):
                bad.append((seed, "bcast", algo, P, dt, nn, o, "errors", rets, st))
        elif any(st) or any(sha(x) != sha(w) for x, w in zip(outs, want)):
            bad.append((seed, "bcast", algo, P, dt, nn, o, "status/data", st))
    rng = random.Random(7000 + seed)
    for _ in range(15):
        coll = rng.choice(R.ROOTED)
        P = rng.choice([1, 2, 3, 4, 4, 6, 8, 8, 16])
        root = 0 if coll == "alltoall" else rng.choice([0, 0, rng.randrange(P)])
        dt = rng.choice(list(F.OPS_OF))
        nn = rng.choice([1, 2, 7, 64, 333, 1000, 4097, rng.randint(1, 20000)])
        flat, relay = rng.random() < 0.4, rng.choice([0, 0, 64, 4096])
        sb = R.inputs(coll, dt, nn, P, seed_base=31 + seed)
        want, exp = R.expect(coll, sb, dt, root, P, nn)
        for c in comms(P):
            c.set_flat_ag(flat)
        outs, st = run_loopback(coll, "bine", sb, dt, root=root, relay=relay)
        nb += 1
        if list(st) != [exp] * P:
            bad.append((seed, coll, P, root, dt, nn, flat, relay, "status", st, exp))
        elif not exp and any(O.canonical(x) != (b"" if w is None else O.canonical(w)) for x, w in zip(outs, want)):
            bad.append((seed, coll, P, root, dt, nn, flat, relay, "data"))
    for PP in (1, 2, 3, 4, 6, 8, 16):
        for c in comms(PP):
            c.set_relay(0); c.set_flat_ag(False)
    print(f"seed {seed}: {nb} bcast / rooted cases, {len(bad)} bad", flush=True)
n += nb
for b in bad[:30]:
    print("BAD", b, flush=True)
print("RESULT", n, "cases", len(bad), "bad", flush=True)
