#!/usr/bin/env python3
"""HBM bytes of the direct transport's collective kernels per process, from
rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes (separate runs) of
tools/dm_tree_ab.py: every rank process of the fused group (it launches
k_dm_move_tree) and of the unfused group (k_reduce_tree), the bytes of
k_dm_move, k_dm_move_tree, k_reduce_tree and k_copy summed per process
(reads = 2 x FETCH_SIZE on gfx950, MI355X_MICROARCH.md "HBM"; writes =
WRITE_SIZE; both in KiB), and the fused / unfused ratio.
usage: python tools/ab_hbm_summary.py FETCH_DIR WRITE_DIR"""
import csv
import glob
import os
import sys

KERNELS = ("k_dm_move_tree", "k_dm_move", "k_reduce_tree", "k_copy")


def short(name):
    return name.split("(")[0].replace("void ", "").split("<")[0].split("::")[-1]


def per_pid(d, counter):
    out = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        pid = os.path.basename(f).split("_")[1] if os.path.basename(f).startswith("ab_") else f
        tot = {}
        for r in csv.DictReader(open(f)):
            if r.get("Counter_Name") != counter:
                continue
            k = short(r["Kernel_Name"])
            if k not in KERNELS:
                continue
            tot[k] = tot.get(k, 0.0) + float(r["Counter_Value"])
        if tot:
            out[pid] = tot
    return out


def main():
    fetch, write = per_pid(sys.argv[1], "FETCH_SIZE"), per_pid(sys.argv[2], "WRITE_SIZE")
    groups = {"fused": [], "unfused": []}
    for pid, f in fetch.items():
        w = write.get(pid)
        # the same pid does not recur across the two passes: match by kernel mix instead
        kind = "fused" if "k_dm_move_tree" in f else "unfused"
        groups[kind].append(f)
    wgroups = {"fused": [w for w in write.values() if "k_dm_move_tree" in w],
               "unfused": [w for w in write.values() if "k_dm_move_tree" not in w]}
    res = {}
    for kind in ("fused", "unfused"):
        rd = sum(2 * sum(f.values()) for f in groups[kind]) * 1024
        wr = sum(sum(w.values()) for w in wgroups[kind]) * 1024
        n = max(len(groups[kind]), 1)
        res[kind] = {"processes": len(groups[kind]), "read_GB_per_process": round(rd / n / 1e9, 3),
                     "write_GB_per_process": round(wr / max(len(wgroups[kind]), 1) / 1e9, 3),
                     "by_kernel_read_GB": {k: round(2 * sum(f.get(k, 0) for f in groups[kind]) * 1024 / n / 1e9, 3)
                                           for k in KERNELS}}
        res[kind]["total_GB_per_process"] = round(res[kind]["read_GB_per_process"] +
                                                  res[kind]["write_GB_per_process"], 3)
    if res["unfused"]["total_GB_per_process"]:
        res["fused_over_unfused"] = round(res["fused"]["total_GB_per_process"] /
                                          res["unfused"]["total_GB_per_process"], 3)
    import json
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
