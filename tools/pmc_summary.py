#!/usr/bin/env python3
"""Summarise rocprofv3 outputs into profiles/<tag>_pmc.json (+ latest_pmc.json).

Inputs (from a GPU run; any depth below each directory):
  gpurun_out/prof/**/*_kernel_trace.csv          rocprofv3 --kernel-trace --stats
  gpurun_out/prof/**/*_kernel_stats.csv          (same pass)
  gpurun_out/pmc_fetch/**/*_counter_collection.csv rocprofv3 --pmc FETCH_SIZE   (own pass)
  gpurun_out/pmc_write/**/*_counter_collection.csv rocprofv3 --pmc WRITE_SIZE   (own pass)
Launches are grouped by (kernel, grid size): one kernel runs at several shapes
in one bench (k_reduce: the C2 launch and the small windows), and the bench's
roofline kernel is the largest-grid shape.  HBM bytes per launch follow
MI355X_MICROARCH.md "HBM": FETCH_SIZE and WRITE_SIZE are in KiB; on gfx950
FETCH_SIZE reads exactly half the bytes of a wide coalesced streaming read, so
reads = 2 * FETCH_SIZE; writes = WRITE_SIZE.
usage: python tools/pmc_summary.py TAG
"""
import csv
import glob
import hashlib
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "gpurun_out")


def short(name):
    return name.split("(")[0].replace("void ", "").split("<")[0].split("::")[-1]


def grid(row):
    for k in ("Grid_Size", "Grid_Size_X", "grid_size"):
        if k in row and row[k] not in (None, ""):
            return int(float(row[k]))
    return 0


def files(sub, suffix):
    return glob.glob(os.path.join(OUT, sub, "**", f"*{suffix}"), recursive=True)


def counters(sub, counter):
    vals = {}
    for path in files(sub, "_counter_collection.csv"):
        for row in csv.DictReader(open(path)):
            if row["Counter_Name"] != counter:
                continue
            vals.setdefault((short(row["Kernel_Name"]), grid(row)), []).append(float(row["Counter_Value"]))
    return vals


def main():
    tag = sys.argv[1] if len(sys.argv) > 1 else "latest"
    trace = {}
    for path in files("prof", "_kernel_trace.csv"):
        for row in csv.DictReader(open(path)):
            k = (short(row["Kernel_Name"]), grid(row))
            ns = float(row["End_Timestamp"]) - float(row["Start_Timestamp"])
            e = trace.setdefault(k, {"name": row["Kernel_Name"], "ns": []})
            e["ns"].append(ns)
    stats = {}
    for path in files("prof", "_kernel_stats.csv"):
        for row in csv.DictReader(open(path)):
            stats[short(row["Name"])] = {"calls": int(row["Calls"]), "avg_ns": float(row["AverageNs"])}
    fetch = counters("pmc_fetch", "FETCH_SIZE")
    write = counters("pmc_write", "WRITE_SIZE")
    shapes = {}
    for k in set(trace) | set(fetch) | set(write):
        e = {}
        if k in trace:
            ns = trace[k]["ns"]
            e.update(name=trace[k]["name"], calls=len(ns), avg_ns=statistics.fmean(ns), median_ns=statistics.median(ns),
                     min_ns=min(ns), max_ns=max(ns))
        if k in fetch:
            e["fetch_size_kib_median"] = statistics.median(fetch[k])
        if k in write:
            e["write_size_kib_median"] = statistics.median(write[k])
        if k in fetch and k in write:
            e["hbm_bytes_per_launch"] = (2 * e["fetch_size_kib_median"] + e["write_size_kib_median"]) * 1024
            e["hbm_bytes_formula"] = "(2*FETCH_SIZE + WRITE_SIZE) KiB, gfx950 FETCH_SIZE correction"
        shapes.setdefault(k[0], {})[k[1]] = e
    kernels = {}
    for name, by_grid in shapes.items():
        g = max(by_grid)
        kernels[name] = dict(by_grid[g], grid_size=g,
                             all_stats_avg_ns=stats.get(name, {}).get("avg_ns"),
                             shapes={str(x): {f: v for f, v in by_grid[x].items() if f != "name"} for x in sorted(by_grid)})
    # the kernel source these counters belong to: bench.py reports `traffic`
    # only while the tree's kernels.hip still hashes to this
    with open(os.path.join(ROOT, "pico_amd", "csrc", "kernels.hip"), "rb") as f:
        src = hashlib.sha256(f.read()).hexdigest()
    res = {"tag": tag, "kernels_hip_sha256": src, "kernels": kernels}
    os.makedirs(os.path.join(ROOT, "profiles"), exist_ok=True)
    for name in (f"{tag}_pmc.json", "latest_pmc.json"):
        with open(os.path.join(ROOT, "profiles", name), "w") as f:
            json.dump(res, f, indent=1)
    print(json.dumps({k: {f: v for f, v in e.items() if f != "shapes"} for k, e in kernels.items()}, indent=1))


if __name__ == "__main__":
    main()
