#!/usr/bin/env python3
"""Search the multi-tree relabellings of pico_amd/csrc/trees.cpp.

For P ranks (power of two) find P-1 permutations sigma_k (sigma_0 = identity)
such that, for every Bine step s, the images sigma_k(M_s) of the step's
pairing M_s = {{r, pi(r, s, P)}} are pairwise edge-disjoint -- P-1 disjoint
perfect matchings of K_P, i.e. every link of a fully connected node once per
step.  Depth-first search with forward filtering; prints the tables.
usage: python tools/find_trees.py [P ...]   (default 4 8)
"""
import itertools
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import oracle as O  # noqa: E402  (pi() of the restatement; host only)


def matchings(P):
    n = P.bit_length() - 1
    return [frozenset(frozenset((r, O.pi(r, s, P))) for r in range(P)) for s in range(n)]


def search(P):
    Ms = matchings(P)
    n = len(Ms)
    perms = list(itertools.permutations(range(P)))

    def image(sig, M):
        return frozenset(frozenset((sig[a], sig[b])) for a, b in (tuple(e) for e in M))

    imgs = [tuple(image(p, M) for M in Ms) for p in perms]
    chosen = [tuple(range(P))]

    def fits(i, used):
        return all(not (imgs[i][s] & used[s]) for s in range(n))

    def rec(cands, used):
        if len(chosen) == P - 1:
            return True
        for idx, i in enumerate(cands):
            nu = [used[s] | imgs[i][s] for s in range(n)]
            nc = [j for j in cands[idx + 1:] if fits(j, nu)]
            chosen.append(perms[i])
            if len(nc) >= P - 1 - len(chosen) and rec(nc, nu):
                return True
            chosen.pop()
        return False

    used = [set(M) for M in Ms]
    ok = rec([i for i in range(len(perms)) if fits(i, used)], used)
    return chosen if ok else None


if __name__ == "__main__":
    for P in [int(x) for x in sys.argv[1:]] or [4, 8]:
        print(P, search(P))
