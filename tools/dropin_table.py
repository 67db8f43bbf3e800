#!/usr/bin/env python3
"""DESIGN.md 4.6's table of libbine.so's default forms (bine_dropin_defaults,
VERDICT r5 item 4): per (P, message size) the node model's time
(pico_amd/model.py) of allreduce_bine_bdw_remap fp32 in the literal schedule
over RCCL P2P (BINE_LITERAL=1) and in the default form (flat phases over the
direct transport, fused trees; one k_dm_fused launch where the plan fits),
and which launch form the default takes.  Host only.
usage: python tools/dropin_table.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pico_amd import model as M  # noqa: E402


def main():
    print("| P | bytes per rank | literal, RCCL (ms) | default (ms) | default launches | speed-up |")
    print("|---|---|---|---|---|---|")
    for P in (2, 4, 8):
        for mib in (1, 16, 64, 256):
            n = (mib << 20) // 4
            # the library's default pipelining chunk: 16 MiB over RCCL, 64 MiB over the direct transport
            lit = M.model_ms("allreduce", "bine_bdw_remap", P, transport="direct", chunk_bytes=16 << 20, count=n)
            dfl = M.model_ms("allreduce", "bine_bdw_remap", P, transport="flatrs+flat+dmt", chunk_bytes=64 << 20,
                             count=n)
            nf = M.fused_launches("allreduce", "bine_bdw_remap", P, transport="flatrs+flat+dmt",
                                  chunk_bytes=64 << 20, count=n)
            form = "1 k_dm_fused" if nf == 1 else f"{dfl['launches']} per-exchange"
            print(f"| {P} | {mib} MiB | {lit['model_ms']:.3f} | {dfl['model_ms']:.3f} | {form} | "
                  f"{lit['model_ms'] / dfl['model_ms']:.1f}x |")


if __name__ == "__main__":
    main()
