#!/usr/bin/env python3
"""Per process of a rocprofv3 kernel trace (one *_kernel_trace.csv per
process): time covered by RCCL's kernels (the exchanges on the comm stream),
by the reduction kernels (k_reduce*, on the compute stream), and by both at
once -- i.e. how much of the reduction work runs while a transfer is in
flight.  usage: python tools/rccl_overlap_report.py <dir>
"""
import csv
import glob
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from overlap_report import intersect, total, union  # noqa: E402


def main():
    d = sys.argv[1]
    for f in sorted(glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)):
        with open(f) as fh:
            ks = list(csv.DictReader(fh))
        red = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in ks if "k_reduce" in r["Kernel_Name"]]
        xch = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in ks if "nccl" in r["Kernel_Name"].lower()]
        if not red or not xch:
            continue
        R, X = union(red), union(xch)
        both = intersect(R, X)
        print(f"{os.path.basename(f)}: reductions {len(red)} launches busy {total(R) / 1e6:.3f} ms; "
              f"RCCL kernels {len(xch)} busy {total(X) / 1e6:.3f} ms; both {both / 1e6:.3f} ms = "
              f"{100 * both / max(1, total(R)):.1f} % of reduction time under a transfer")


if __name__ == "__main__":
    main()
