#!/usr/bin/env python3
"""Summarise a rocprofv3 kernel + memory-copy trace of tools/overlap_probe.py:
time covered by reduction kernels, by exchange traffic (copy kernels / SDMA
copies), and by both at once.  usage: python tools/overlap_report.py <dir>
"""
import csv
import glob
import os
import sys


def rows(pattern):
    out = []
    for f in glob.glob(pattern, recursive=True):
        with open(f) as fh:
            out += list(csv.DictReader(fh))
    return out


def union(iv):
    iv = sorted(iv)
    out = []
    for a, b in iv:
        if out and a <= out[-1][1]:
            out[-1][1] = max(out[-1][1], b)
        else:
            out.append([a, b])
    return out


def total(u):
    return sum(b - a for a, b in u)


def intersect(u, v):
    i = j = 0
    t = 0
    while i < len(u) and j < len(v):
        a, b = max(u[i][0], v[j][0]), min(u[i][1], v[j][1])
        if a < b:
            t += b - a
        if u[i][1] < v[j][1]:
            i += 1
        else:
            j += 1
    return t


def main():
    d = sys.argv[1]
    ks = rows(os.path.join(d, "**", "*kernel_trace.csv"))
    ms = rows(os.path.join(d, "**", "*memory_copy_trace.csv"))
    red = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in ks if "k_reduce" in r["Kernel_Name"]]
    cpk = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in ks
           if "k_reduce" not in r["Kernel_Name"] and "fill" not in r["Kernel_Name"]]
    cps = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in ms]
    R, X = union(red), union(cpk + cps)
    span = (max(b for _, b in R + X) - min(a for a, _ in R + X)) if R and X else 0
    print(f"reduction kernels: {len(red)} launches, busy {total(R) / 1e6:.3f} ms")
    print(f"exchange copies:   {len(cpk)} copy kernels + {len(cps)} SDMA copies, busy {total(X) / 1e6:.3f} ms")
    print(f"both at once:      {intersect(R, X) / 1e6:.3f} ms "
          f"({100 * intersect(R, X) / max(1, total(R)):.1f} % of reduction time overlapped)")
    print(f"trace span:        {span / 1e6:.3f} ms")


if __name__ == "__main__":
    main()
