#!/usr/bin/env python3
"""End-to-end rate with host buffers (north_star: "the end-to-end rate
including H2D and D2H copies"): the reference's UNCHANGED pico_core
(integration/_build/pico_core) through libbine.so, allreduce
bine_bdw_remap_over, 256 MiB per rank, host (malloc) buffers -- per
configuration the median of pico_core's own per-iteration times (its CSV,
max over ranks, first 20 % dropped), every iteration checked by pico_core
against PMPI_Allreduce.  Configurations: the staging pipeline's chunk
(BINE_STAGE_CHUNK_BYTES) and per-call page-locking on / off (BINE_HOST_REGISTER).
Configuration set "pipeline" (5th argument; floating point at P > 1): the
serial path (BINE_STAGE_PIPELINE=0: H2D, then the collective, then D2H)
against the staging pipelined into the collective (bine_allreduce_staged)
at several chunks.
Configuration set "c1" (BASELINE config C1: 262,144 fp32 per rank at P = 4,
the reference's own CPU-runnable case): the transports libbine.so offers --
RCCL, RCCL with the flat phases, the direct transport, the direct transport
with the flat phases (one k_dm_fused launch per call).
usage: python tools/e2e_staging.py [NP] [DTYPE] [COUNT] [ITERS] [chunks|pipeline|c1|zc]"""
import json
import os
import statistics
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run(np_, dtype, count, iters, env_extra):
    with tempfile.TemporaryDirectory() as tmp:
        env = dict(os.environ, PICO_OUT=tmp, **env_extra)
        if np_ > 1:
            env["BINE_FAKE_HOSTS"] = "1"
        p = subprocess.run(["bash", os.path.join(ROOT, "integration", "run_pico_core.sh"), str(np_), "ALLREDUCE",
                            str(count), str(iters), "bine_bdw_remap_over", dtype], env=env, capture_output=True,
                           text=True, timeout=300)
        if p.returncode != 0:
            return {"error": (p.stdout[-400:] + p.stderr[-400:])}
        rows = open(os.path.join(tmp, "data", f"{count}_bine_bdw_remap_over_{dtype}.csv")).read().splitlines()[1:]
        hi = [float(r.split(",")[0]) * 1e-6 for r in rows]   # ns -> ms
        kept = hi[int(len(hi) * 0.2):]
        return {"ms_median": round(statistics.median(kept), 4), "ms_min": round(min(kept), 4), "iters": len(hi),
                "pico_core_check": "passed"}


if __name__ == "__main__":
    np_ = int(sys.argv[1]) if len(sys.argv) > 1 else 1
    dtype = sys.argv[2] if len(sys.argv) > 2 else "float"
    count = int(sys.argv[3]) if len(sys.argv) > 3 else 67108864
    iters = int(sys.argv[4]) if len(sys.argv) > 4 else 20
    esz = {"float": 4, "double": 8, "int64": 8, "int32": 4}[dtype]
    S = count * esz
    out = {"np": np_, "dtype": dtype, "count": count, "bytes_per_rank": S}
    # host buffers page-locked per call (registered at the start of each call,
    # unregistered before it returns; round 4) or pageable (HIP's own staging)
    cfgs = [("pageable, one collective", {"BINE_HOST_REGISTER": "0", "BINE_STAGE_CHUNK_BYTES": str(1 << 40)}),
            ("page-locked per call, one collective", {"BINE_STAGE_CHUNK_BYTES": str(1 << 40)}),
            ("pageable, 16 MiB chunks", {"BINE_HOST_REGISTER": "0"}),
            ("page-locked per call, 8 MiB chunks", {"BINE_STAGE_CHUNK_BYTES": str(8 << 20)}),
            ("page-locked per call, 16 MiB chunks (default)", {}),
            ("page-locked per call, 32 MiB chunks", {"BINE_STAGE_CHUNK_BYTES": str(32 << 20)})]
    if len(sys.argv) > 5 and sys.argv[5] == "pipeline":
        cfgs = [("serial: H2D, collective, D2H (BINE_STAGE_PIPELINE=0)", {"BINE_STAGE_PIPELINE": "0"}),
                ("pipelined into the collective, 16 MiB rounds (default)", {}),
                ("pipelined, 4 MiB rounds", {"BINE_STAGE_CHUNK_BYTES": str(4 << 20)}),
                ("pipelined, 8 MiB rounds", {"BINE_STAGE_CHUNK_BYTES": str(8 << 20)}),
                ("pipelined, 32 MiB rounds", {"BINE_STAGE_CHUNK_BYTES": str(32 << 20)}),
                ("pipelined, 64 MiB rounds", {"BINE_STAGE_CHUNK_BYTES": str(64 << 20)})]
        out["transport"] = "direct peer memory (BINE_DIRECT=1)" if os.environ.get("BINE_DIRECT") == "1" else "RCCL"
    if len(sys.argv) > 5 and sys.argv[5] == "c1":
        # round 6: libbine.so's defaults (bine_dropin_defaults: flat phases over the
        # direct transport, one k_dm_fused launch; host buffers page-locked per
        # call) against the variants: bounce buffers, pageable, RCCL, literal
        cfgs = [("default (no BINE_* setting): flat phases, direct transport, host buffers in place (zero copy)", {}),
                ("default forms, staged through device buffers (BINE_HOST_ZERO_COPY_BYTES=0)",
                 {"BINE_HOST_ZERO_COPY_BYTES": "0"}),
                ("default forms, bounce buffers (BINE_HOST_BOUNCE_BYTES=4 MiB)", {"BINE_HOST_BOUNCE_BYTES": str(4 << 20)}),
                ("default forms, pageable (HIP's own staging)", {"BINE_HOST_REGISTER": "0"}),
                ("flat phases over RCCL (BINE_DIRECT=0)", {"BINE_DIRECT": "0"}),
                ("literal schedule over RCCL (BINE_LITERAL=1, round 5's default)", {"BINE_LITERAL": "1"})]
    if len(sys.argv) > 5 and sys.argv[5] == "zc":
        # the zero-copy threshold (BINE_HOST_ZERO_COPY_BYTES): the default forms
        # with the host buffers addressed in place vs staged through device buffers
        cfgs = [("zero copy (BINE_HOST_ZERO_COPY_BYTES=1 GiB)", {"BINE_HOST_ZERO_COPY_BYTES": str(1 << 30)}),
                ("staged (BINE_HOST_ZERO_COPY_BYTES=0)", {"BINE_HOST_ZERO_COPY_BYTES": "0"})]
    for name, env in cfgs:
        r = run(np_, dtype, count, iters, env)
        if "ms_median" in r:
            r["algbw_GBs"] = round(S / (r["ms_median"] * 1e-3) / 1e9, 2)
            r["pcie_bytes_GBs"] = round(2 * S / (r["ms_median"] * 1e-3) / 1e9, 2)
        out[name] = r
        print(name, json.dumps(r), flush=True)
    print(json.dumps(out))
