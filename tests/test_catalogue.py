"""config/algorithm_config_mi355x.json (tools/make_catalogue.py): every entry
resolves to a library algorithm through pico_core's selector string, and its
comm_sz constraints are exactly the sizes the planner accepts (P = 1 ... 16; root 0,
pico_core's), so
the reference's parse_test.py never schedules a run the library refuses."""
import json
import os

import pico_amd

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CAT = os.path.join(ROOT, "config", "algorithm_config_mi355x.json")


def _ok(cons, P):
    for c in cons:
        if c["key"] != "comm_sz":
            continue
        for cond in c["conditions"]:
            op, v = cond["operator"], cond["value"]
            if op == "is_power_of_two" and P & (P - 1):
                return False
            if op == "is_even" and P % 2:
                return False
            if op == ">=" and not P >= v:
                return False
    return True


def test_catalogue_is_current():
    import importlib.util
    spec = importlib.util.spec_from_file_location("mk", os.path.join(ROOT, "tools", "make_catalogue.py"))
    mk = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mk)
    assert json.load(open(CAT)) == json.loads(json.dumps(mk.catalogue()))


def test_entries_resolve_and_constraints_match_planner():
    cat = json.load(open(CAT))["collective"]
    lib = pico_amd.lib()
    n = 0
    for coll, entries in cat.items():
        c = coll.lower()
        for sel, e in entries.items():
            algo = lib.bine_algo_from_name(c.encode(), sel.encode())
            assert algo == pico_amd.ALGOS[c][e["tags"][0]], (coll, sel)
            assert "cuda" in e["tags"]
            for P in range(1, 17):
                try:
                    pico_amd.plan(c, algo, P, 0, count=4 * P, rcounts=[4] * P)
                    planned = True
                except pico_amd.BineError:
                    planned = False
                allowed = _ok(e.get("constraints", []), P)
                # the catalogue may only be stricter, and only at P = 1 (is_even
                # rules out the single-rank copy of reduce_scatter any_even)
                assert planned == allowed or (P == 1 and planned and not allowed), (coll, sel, P)
            n += 1
    assert n == 41   # 8 + 9 + 2 reduce family, 12 allgather, 7 bcast, alltoall, gather, scatter
