#!/usr/bin/env python3
"""Write config/algorithm_config_mi355x.json: the MI355X library's algorithms as
entries of the reference's test catalogue (config/algorithm_config.json
schema: desc / library / cvar / dynamic_rule / constraints / tags), so the
reference's parse_test.py (:116-185) selects them -- the "cuda" tag is what it
requires under GPU_AWARENESS=yes (:141-142), "is_segmented" marks the segmented
variant (:170-173).  Entry names are pico_core's selector strings
(pico_core_utils.c:103-249); constraints are the ones this library enforces
(checked against the planner by tests/test_catalogue.py).
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

POW2 = {"key": "comm_sz", "conditions": [{"operator": "is_power_of_two", "value": True}]}
POW2_MIN2 = {"key": "comm_sz", "conditions": [{"operator": "is_power_of_two", "value": True},
                                               {"operator": ">=", "value": 2}]}
EVEN = {"key": "comm_sz", "conditions": [{"operator": "is_even", "value": True}]}
COUNT_GE_P = {"key": "count", "conditions": [{"operator": ">=", "value": "comm_sz"}]}

# (collective, libbine short name, selector, constraints, extra tags, description)
ENTRIES = [
    ("ALLREDUCE", "recursivedoubling", "recursive_doubling_over", [], ["latency_optimal"],
     "Recursive doubling (libbine_allreduce.c:17)."),
    ("ALLREDUCE", "ring", "ring_over", [], ["bandwidth_optimal", "ring"], "Ring reduce-scatter + allgather (:138)."),
    ("ALLREDUCE", "rabenseifner", "rabenseifner_over", [], ["bandwidth_optimal"], "Rabenseifner (:441)."),
    ("ALLREDUCE", "bine_lat", "bine_lat_over", [], ["bine", "latency_optimal"], "Bine latency-optimal (:321)."),
    ("ALLREDUCE", "bine_bdw_static", "bine_bdw_static_over", [POW2_MIN2], ["bine", "bandwidth_optimal", "static"],
     "Bine bandwidth-optimal, static tables (:696)."),
    ("ALLREDUCE", "bine_bdw_remap", "bine_bdw_remap_over", [POW2], ["bine", "bandwidth_optimal", "remap"],
     "Bine bandwidth-optimal, remapped contiguous windows (:820). Headline path."),
    ("ALLREDUCE", "bine_bdw_remap_segmented", "bine_bdw_remap_segmented_over", [],
     ["bine", "bandwidth_optimal", "remap", "is_segmented"], "Bine remap with segment pipelining (:1093)."),
    ("ALLREDUCE", "bine_block_by_block_any_even", "bine_block_by_block_any_even", [EVEN],
     ["bine", "bandwidth_optimal", "block_by_block"], "Bine block-by-block, any even size (:925)."),
    ("REDUCE_SCATTER", "recursivehalving", "recursive_halving_over", [], ["bandwidth_optimal"],
     "Recursive halving (libbine_reduce_scatter.c:15)."),
    ("REDUCE_SCATTER", "recursive_distance_doubling", "recursive_distance_doubling_over", [POW2],
     ["bandwidth_optimal"], "Recursive distance doubling (:259)."),
    ("REDUCE_SCATTER", "ring", "ring_over", [], ["bandwidth_optimal", "ring"], "Ring (:421)."),
    ("REDUCE_SCATTER", "butterfly", "butterfly_over", [], ["bandwidth_optimal"], "Butterfly (:575)."),
    ("REDUCE_SCATTER", "bine_static", "bine_static_over", [POW2_MIN2], ["bine", "bandwidth_optimal", "static"],
     "Bine, static tables (:763)."),
    ("REDUCE_SCATTER", "bine_send_remap", "bine_send_remap_over", [POW2], ["bine", "bandwidth_optimal", "remap"],
     "Bine remap with a final send (:906)."),
    ("REDUCE_SCATTER", "bine_permute_remap", "bine_permute_remap_over", [POW2],
     ["bine", "bandwidth_optimal", "remap"], "Bine remap with an initial local permutation (:985)."),
    ("REDUCE_SCATTER", "bine_block_by_block", "bine_block_by_block_over", [POW2],
     ["bine", "bandwidth_optimal", "block_by_block"], "Bine block-by-block (:1066)."),
    ("REDUCE_SCATTER", "bine_block_by_block_any_even", "bine_block_by_block_any_even", [EVEN],
     ["bine", "bandwidth_optimal", "block_by_block"], "Bine block-by-block, any even size (:1176)."),
    ("REDUCE", "bine_lat", "bine_lat_over", [POW2], ["bine", "latency_optimal"], "Bine binomial (libbine_reduce.c:16)."),
    ("REDUCE", "bine_bdw", "bine_bdw_over", [POW2], ["bine", "bandwidth_optimal"], "Bine RS + gather (:83)."),
    ("ALLGATHER", "k_bruck", "k_bruck_over", [], ["latency_optimal"], "Bruck, radix 2 (libbine_allgather.c:88)."),
    ("ALLGATHER", "recursivedoubling", "recursive_doubling_over", [POW2], ["latency_optimal"],
     "Recursive doubling (:18)."),
    ("ALLGATHER", "ring", "ring_over", [], ["bandwidth_optimal", "ring"], "Ring (:213)."),
    ("ALLGATHER", "sparbit", "sparbit_over", [], ["latency_optimal"], "Sparbit (:327)."),
    ("ALLGATHER", "bine_block_by_block_any_even", "bine_block_by_block_over_any_even", [EVEN],
     ["bine", "block_by_block"], "Bine block-by-block, any even size (:492)."),
    ("ALLGATHER", "bine_block_by_block", "bine_block_by_block_over", [POW2_MIN2], ["bine", "block_by_block"],
     "Bine block-by-block (:410)."),
    ("ALLGATHER", "bine_permute_static", "bine_permute_static_over", [POW2_MIN2], ["bine", "static"],
     "Bine static, final permutation folded into placement (:563)."),
    ("ALLGATHER", "bine_send_static", "bine_send_static_over", [POW2_MIN2], ["bine", "static"],
     "Bine static, initial send (:642)."),
    ("ALLGATHER", "bine_permute_remap", "bine_permute_remap_over", [POW2_MIN2], ["bine", "remap"],
     "Bine remap, final permutation folded into placement (:725)."),
    ("ALLGATHER", "bine_send_remap", "bine_send_remap_over", [POW2_MIN2], ["bine", "remap"],
     "Bine remap, initial send (:811)."),
    ("ALLGATHER", "bine_2_blocks", "bine_2_blocks_over", [POW2_MIN2], ["bine"], "Bine two-block (:892)."),
    ("ALLGATHER", "bine_2_blocks_dtype", "bine_2_blocks_dtype_over", [POW2_MIN2], ["bine"],
     "Bine two-block, derived-datatype variant (:999)."),
    ("BCAST", "bine_lat", "bine_lat_over", [POW2], ["bine", "latency_optimal"],
     "Bine binomial tree, root 0 (libbine_bcast.c:189)."),
    ("BCAST", "bine_lat_reversed", "bine_lat_reversed_over", [POW2], ["bine", "latency_optimal"],
     "Bine binomial tree, steps reversed, root 0 (:281)."),
    ("BCAST", "bine_lat_new", "bine_lat_new_over", [POW2], ["bine", "latency_optimal"],
     "Bine binomial tree, negabinary partners, any root (:373)."),
    ("BCAST", "bine_lat_i_new", "bine_lat_i_new_over", [POW2], ["bine", "latency_optimal"],
     "Bine binomial tree, negabinary partners, non-blocking sends (:408)."),
    ("BCAST", "scatter_allgather", "scatter_allgather_over", [COUNT_GE_P], ["bandwidth_optimal"],
     "Binomial scatter + recursive-doubling allgather (:42)."),
    ("BCAST", "bine_bdw_static", "bine_bdw_static_over", [POW2, COUNT_GE_P], ["bine", "bandwidth_optimal", "static"],
     "Bine static-table scatter + allgather, root 0 (:462)."),
    ("BCAST", "bine_bdw_remap", "bine_bdw_remap_over", [POW2], ["bine", "bandwidth_optimal", "remap"],
     "Bine remapped scatter + allgather, root 0 (:649)."),
    ("ALLTOALL", "bine", "bine_over", [POW2], ["bine"], "Bine butterfly (libbine_alltoall.c:14)."),
    ("GATHER", "bine", "bine_over", [POW2], ["bine"],
     "Bine tree, root 0 and the even roots the reference serves (libbine_gather.c:16)."),
    ("SCATTER", "bine", "bine_over", [POW2], ["bine"],
     "Bine tree, root 0 and the roots the reference serves (libbine_scatter.c:14)."),
]


def catalogue():
    out = {"config_metadata": {
        "schema_version": "2.6.15",
        "description": "MI355X library (libbine.so drop-in over RCCL/xGMI with CDNA4 reduction kernels): "
                       "entries in the schema of the reference's config/algorithm_config.json",
        "generator": "tools/make_catalogue.py"},
        "collective": {}}
    for coll, name, sel, cons, tags, desc in ENTRIES:
        e = {"desc": desc + " MI355X: device buffers, RCCL P2P, HIP reduction kernels.",
             "library": {"libbine": "1.0.0"}, "cvar": "auto", "dynamic_rule": 0,
             "tags": [name, "external", "cuda", "mi355x", "rccl"] + tags}
        if cons:
            e["constraints"] = cons
        out["collective"].setdefault(coll, {})[sel] = e
    return out


if __name__ == "__main__":
    os.makedirs(os.path.join(ROOT, "config"), exist_ok=True)
    path = os.path.join(ROOT, "config", "algorithm_config_mi355x.json")
    with open(path, "w") as f:
        json.dump(catalogue(), f, indent=2)
        f.write("\n")
    print(path)
