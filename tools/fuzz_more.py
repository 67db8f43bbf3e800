"""The GPU fuzz of tests/test_gpu_fuzz.py over more seeds than the suite runs
(seeds 100 ... 100 + N - 1, 60 random configurations each: collective x
algorithm x P x count x type x operator x transport setting x in place on
loopback ranks, bit-exact vs the oracle or the expected error).
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
for b in bad[:30]:
    print("BAD", b, flush=True)
print("RESULT", n, "cases", len(bad), "bad", flush=True)
