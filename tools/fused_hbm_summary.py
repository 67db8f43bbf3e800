#!/usr/bin/env python3
"""HBM bytes of the one-launch direct-transport collectives (k_dm_fused) on
one GPU shared by two rank processes, from separate rocprofv3 --pmc
FETCH_SIZE / WRITE_SIZE passes of tools/dm_stamps.py 2 ITERS (VERDICT r4
item 4).

The TCC counters are device-wide, so a process's per-dispatch sample also
counts the peer's traffic while the two kernels run together -- which they
must: each waits for the other's flags.  With the whole call in ONE launch
per rank the two windows nearly coincide, so each sample is the bytes of
BOTH ranks' calls (the device-wide window); the window overlap is measured
from the dispatch timestamps and printed beside it.  The figure compared
with pico_amd/model.py is therefore: device bytes per call (median over the
timed calls of the two processes' mean sample) / (2 x the model's bytes per
rank).  reads = 2 x FETCH_SIZE on gfx950 (MI355X_MICROARCH.md "HBM"),
writes = WRITE_SIZE, both in KiB.

dm_stamps.py runs C3 (1 + ITERS calls, one launch each) then C4 (1 + ITERS
calls, launches per call from the model) per process.
usage: python tools/fused_hbm_summary.py FETCH_DIR WRITE_DIR ITERS
"""
import csv
import glob
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def dispatches(d, counter):
    """per process: [(value_KiB, start, end)] of k_dm_fused in dispatch order"""
    out = []
    for f in sorted(glob.glob(os.path.join(d, "*counter_collection.csv"))):
        rows = [r for r in csv.DictReader(open(f)) if r["Counter_Name"] == counter and "k_dm_fused" in r["Kernel_Name"]]
        rows.sort(key=lambda r: int(r["Dispatch_Id"]))
        out.append([(float(r["Counter_Value"]), int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows])
    return out


def overlap(a, b):
    lo, hi = max(a[1], b[1]), min(a[2], b[2])
    return max(0, hi - lo) / (max(a[2], b[2]) - min(a[1], b[1]))


def main():
    fdir, wdir, iters = sys.argv[1], sys.argv[2], int(sys.argv[3])
    from pico_amd import model as M
    F, W = dispatches(fdir, "FETCH_SIZE"), dispatches(wdir, "WRITE_SIZE")
    assert len(F) == 2 and len(W) == 2, (len(F), len(W))
    c3_l = M.config_model("C3", 2, "flatrs+flat+dmt", 64 << 20)["launches"]
    c4_l = M.config_model("C4", 2, "flatrs+flat+dmt", 64 << 20)["launches"]
    res = {}
    start = 0
    for cfg, nl in (("C3", c3_l), ("C4", c4_l)):
        per_call, ov = [], []
        for k in range(1 + iters):
            sl = slice(start + k * nl, start + (k + 1) * nl)
            if k == 0:
                continue   # the warm-up call
            rd = [2 * sum(v for v, _, _ in F[p][sl]) * 1024 for p in range(2)]
            wr = [sum(v for v, _, _ in W[p][sl]) * 1024 for p in range(2)]
            per_call.append((sum(rd) / 2, sum(wr) / 2))
            ov += [overlap(a, b) for a, b in zip(F[0][sl], F[1][sl])] + [overlap(a, b) for a, b in zip(W[0][sl], W[1][sl])]
        start += (1 + iters) * nl
        model = M.config_model(cfg, 2, "flatrs+flat+dmt", 64 << 20)["hbm_bytes"]
        rd = statistics.median(x for x, _ in per_call)
        wr = statistics.median(y for _, y in per_call)
        res[cfg] = {"launches_per_call": nl, "device_read_GB_per_call": round(rd / 1e9, 4),
                    "device_write_GB_per_call": round(wr / 1e9, 4),
                    "device_GB_per_call": round((rd + wr) / 1e9, 4),
                    "model_GB_per_call_both_ranks": round(2 * model / 1e9, 4),
                    "measured_over_model": round((rd + wr) / (2 * model), 4),
                    "window_overlap_median": round(statistics.median(ov), 4),
                    "window_overlap_min": round(min(ov), 4)}
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
