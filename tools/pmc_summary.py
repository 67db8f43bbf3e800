#!/usr/bin/env python3
"""Summarise rocprofv3 outputs into profiles/<tag>_pmc.json (+ latest_pmc.json).

Inputs (from a GPU run, see DESIGN.md "Measurement"):
  gpurun_out/prof/*_kernel_stats.csv           rocprofv3 --kernel-trace --stats
  gpurun_out/pmc_fetch/*_counter_collection.csv rocprofv3 --pmc FETCH_SIZE   (own pass)
  gpurun_out/pmc_write/*_counter_collection.csv rocprofv3 --pmc WRITE_SIZE   (own pass)
HBM bytes per launch follow MI355X_MICROARCH.md "HBM": FETCH_SIZE and WRITE_SIZE
are in KiB; on gfx950 FETCH_SIZE reads exactly half the bytes of a wide
coalesced streaming read, so reads = 2 * FETCH_SIZE; writes = WRITE_SIZE.
usage: python tools/pmc_summary.py TAG
"""
import csv
import glob
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "gpurun_out")


def short(name):
    return name.split("(")[0].replace("void ", "").split("<")[0].split("::")[-1]


def counters(pattern, counter):
    vals = {}
    for path in glob.glob(os.path.join(OUT, pattern)):
        for row in csv.DictReader(open(path)):
            if row["Counter_Name"] != counter:
                continue
            vals.setdefault(short(row["Kernel_Name"]), []).append(float(row["Counter_Value"]))
    return vals


def main():
    tag = sys.argv[1] if len(sys.argv) > 1 else "latest"
    stats = {}
    for path in glob.glob(os.path.join(OUT, "prof", "*_kernel_stats.csv")):
        for row in csv.DictReader(open(path)):
            stats[short(row["Name"])] = {"name": row["Name"], "calls": int(row["Calls"]),
                                         "avg_ns": float(row["AverageNs"]), "min_ns": float(row["MinNs"]),
                                         "max_ns": float(row["MaxNs"])}
    fetch = counters("pmc_fetch/*_counter_collection.csv", "FETCH_SIZE")
    write = counters("pmc_write/*_counter_collection.csv", "WRITE_SIZE")
    kernels = {}
    for k in set(stats) | set(fetch) | set(write):
        e = dict(stats.get(k, {}))
        if k in fetch:
            e["fetch_size_kib_median"] = statistics.median(fetch[k])
        if k in write:
            e["write_size_kib_median"] = statistics.median(write[k])
        if k in fetch and k in write:
            e["hbm_bytes_per_launch"] = (2 * e["fetch_size_kib_median"] + e["write_size_kib_median"]) * 1024
            e["hbm_bytes_formula"] = "(2*FETCH_SIZE + WRITE_SIZE) KiB, gfx950 FETCH_SIZE correction"
        kernels[k] = e
    res = {"tag": tag, "kernels": kernels}
    os.makedirs(os.path.join(ROOT, "profiles"), exist_ok=True)
    for name in (f"{tag}_pmc.json", "latest_pmc.json"):
        with open(os.path.join(ROOT, "profiles", name), "w") as f:
            json.dump(res, f, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
