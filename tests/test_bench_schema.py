"""bench.py's N > 1 JSON line and its error agreement, host logic only
(VERDICT r5 item 5 / weak #6, item 1's consequences for the bench):

* ranks sharing ONE GPU (BINE_FAKE_HOSTS=1, the one-GPU rehearsal): the
  roofline names the bound in play -- the one HBM, every rank's bytes of the
  executed schedule -- with frac <= 1, the xGMI roofline kept for a node;
  on a node (no BINE_FAKE_HOSTS) the roofline is the link's;
* the node model recomputed from the direct-transport probe's measured
  constants;
* a library error seen on ONE rank (a direct-transport wait that timed out is
  reported at the completion of the call on the rank that timed out) is
  agreed over all ranks, so every rank takes the same branch and the ranks
  never wait in different collectives (gloo, 2 processes)."""
import os
import socket
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import pico_amd  # noqa: E402

ST = {"median_ms": 0.45, "mean_ms": 0.46, "min_ms": 0.44, "max_ms": 0.5, "samples": 4, "region_ms": 0.46,
      "issue_ms": 0.01, "wall_s": 0.1}
CFG = ("flatrs+flat+dmt", 64 << 20, False)


def _line(monkeypatch, fake_hosts):
    if fake_hosts:
        monkeypatch.setenv("BINE_FAKE_HOSTS", "1")
    else:
        monkeypatch.delenv("BINE_FAKE_HOSTS", raising=False)
    key = bench.gkey("C3", "allreduce", "bine_bdw_remap", "float", bench.C3_ELEMS, 2)
    return bench._headline_line(pico_amd, "bine_bdw_remap", 2, 0, bench.C3_ELEMS, 5, 1, key, CFG, ST, True, 1,
                                None, {CFG: 0.45}, {CFG: True})


def test_one_gpu_rehearsal_roofline_is_the_hbm(monkeypatch):
    d = _line(monkeypatch, True)
    r = d["roofline"]
    assert r["bound"] == "hbm" and r["unit"] == "GB/s" and r["peak"] == bench.HBM_PEAK_GBS
    # C3 at P = 2, one k_dm_fused launch per call: 4.0 S per rank (pico_amd/model.py)
    S = bench.C3_ELEMS * 4
    assert r["algorithmic_bytes_per_call"] == 2 * 4 * S
    assert r["achieved"] == pytest.approx(2 * 4 * S / 0.45e-3 / 1e9, rel=1e-3)
    assert 0 < r["frac"] <= 1
    link = r["link_roofline_if_node"]
    assert link["bound"] == "xgmi" and link["link_time_bytes"] > 0 and "model" not in link
    assert r["model_ms"] > 0 and r["model"]["one_gpu"] is True
    assert d["metric"] == bench.METRIC and d["n_gpus"] == 2 and d["value"] > 0


def test_node_roofline_is_the_link(monkeypatch):
    r = _line(monkeypatch, False)["roofline"]
    assert r["bound"] == "xgmi" and "link_roofline_if_node" not in r
    # flat RS + flat AG at P = 2: every op loads the one link, so peak = 153 GB/s
    assert r["peak"] == pytest.approx(bench.XGMI_LINK_GBS)
    assert r["model"]["one_gpu"] is False


def test_model_with_measured_constants(monkeypatch):
    monkeypatch.delenv("BINE_FAKE_HOSTS", raising=False)
    from pico_amd import model as M
    base = bench.measured_models(8, "flatrs+flat+dmt", 64 << 20, M.LINK_GBS, M.T_FLAG_US)
    slow = bench.measured_models(8, "flatrs+flat+dmt", 64 << 20, M.LINK_GBS / 2, 2 * M.T_FLAG_US)
    assert base["C3"] == bench.node_model("C3", 8, "flatrs+flat+dmt", 64 << 20)["model_ms"]
    assert base["C1_e2e_us"] == M.c1_e2e_us(8)["e2e_us"]
    assert slow["C3"] > base["C3"] and slow["C4"] > base["C4"] and slow["C1_e2e_us"] > base["C1_e2e_us"]
    # ranks sharing one GPU: the push figure is no link rate -- C1 keeps the assumed link rate
    monkeypatch.setenv("BINE_FAKE_HOSTS", "1")
    one = bench.measured_models(8, "flatrs+flat+dmt", 64 << 20, 0.41, M.T_FLAG_US)
    assert one["one_gpu"] and one["C1_e2e_us"] == M.c1_e2e_us(8)["e2e_us"] and "C1_note" in one


class _Comm:
    """a communicator whose completion fails on one rank only"""
    def __init__(self, bad):
        self.bad = bad

    def synchronize(self):
        if self.bad:
            raise pico_amd.BineError(7, "bine_comm_synchronize")


def _agree_worker(rank, port, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=2)
    # completion error on rank 1 only
    d = bench.Drain(_Comm(rank == 1))
    d()
    a = d.failed(dist)
    # issue-time error on rank 0 only: nothing more is issued there
    calls = []

    def call():
        calls.append(1)
        if rank == 0:
            raise pico_amd.BineError(7, "bine_allreduce")
    d2 = bench.Drain(_Comm(False))
    g = d2.guard(call)
    g()
    g()
    d2()
    b = d2.failed(dist)
    d3 = bench.Drain(_Comm(False))
    d3()
    c = d3.failed(dist)
    dist.destroy_process_group()
    q.put((rank, a, b, c, len(calls)))


def test_library_errors_agreed_over_ranks():
    import multiprocessing as mp
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_agree_worker, args=(r, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = dict((o[0], o[1:]) for o in (q.get(timeout=120) for _ in ps))
    for p in ps:
        p.join(30)
    assert all(p.exitcode == 0 for p in ps)
    for r in (0, 1):
        a, b, c, ncalls = res[r]
        assert a is not None and a.startswith("rank 1: ") and "KFD compute queues" in a and "rank 0:" not in a
        assert b is not None and b.startswith("rank 0: ")
        assert c is None
        assert ncalls == (1 if r == 0 else 2)
