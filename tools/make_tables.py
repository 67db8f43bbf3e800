#!/usr/bin/env python3
"""Digest the reference's static Bine tables (test infrastructure).

Parses /root/reference/libbine/libbine_utils_bitmaps.c (perm_P, remap_P,
send_P, recv_P for P = 2..256) and writes tests/golden/tables.json holding, per
P, the SHA-256 of each table as little-endian int32 (row-major), plus the
tables themselves for P <= 8.  tests/test_oracle.py checks the oracle's and the
product planner's generated tables against these digests (and against the
source itself when /root/reference is present).
"""
import hashlib
import json
import os
import re

import numpy as np

SRC = "/root/reference/libbine/libbine_utils_bitmaps.c"
OUT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden", "tables.json")


def parse(src=SRC):
    text = open(src).read()
    tabs = {}
    for m in re.finditer(r"const int (perm|remap|send|recv)_(\d+)(?:\[\d+\])+\s*=\s*\{(.*?)\};", text, re.S):
        kind, P, body = m.group(1), int(m.group(2)), m.group(3)
        vals = [int(x) for x in re.findall(r"-?\d+", body)]
        tabs[(kind, P)] = np.array(vals, dtype="<i4")
    return tabs


def digest(a):
    return hashlib.sha256(np.asarray(a, dtype="<i4").tobytes()).hexdigest()


def main():
    tabs = parse()
    out = {}
    for (kind, P), a in sorted(tabs.items()):
        e = out.setdefault(str(P), {})
        e[kind + "_sha256"] = digest(a)
        if P <= 8:
            e[kind] = a.tolist()
    json.dump({"source": "libbine/libbine_utils_bitmaps.c:10-56", "tables": out}, open(OUT, "w"), indent=1)
    print(len(tabs), "tables")


if __name__ == "__main__":
    main()
