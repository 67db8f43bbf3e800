#!/usr/bin/env python3
"""Per-process kernel summary of rocprofv3 --kernel-trace CSVs under a
directory: for every *_kernel_trace.csv, each kernel's launch count, median /
mean / total duration (us), and the busy span of the file.
usage: python tools/trace_summary.py DIR [KERNEL_SUBSTRING ...]
"""
import csv
import glob
import os
import statistics
import sys


def short(name):
    base = name.split("(")[0].replace("void ", "")
    return base.replace("bine::", "")


def main():
    d = sys.argv[1]
    keep = sys.argv[2:]
    for f in sorted(glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)):
        rows = list(csv.DictReader(open(f)))
        if not rows:
            continue
        by = {}
        t0 = min(int(r["Start_Timestamp"]) for r in rows)
        t1 = max(int(r["End_Timestamp"]) for r in rows)
        for r in rows:
            k = short(r["Kernel_Name"])
            if keep and not any(s in k for s in keep):
                continue
            by.setdefault(k, []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
        print(f"## {os.path.relpath(f, d)}: {len(rows)} kernels, span {(t1 - t0) / 1e6:.1f} ms")
        for k, v in sorted(by.items(), key=lambda kv: -sum(kv[1])):
            print(f"  {len(v):6d}  median {statistics.median(v):10.1f} us  mean {statistics.mean(v):10.1f} us  "
                  f"total {sum(v) / 1e3:9.2f} ms  {k}")


if __name__ == "__main__":
    main()
