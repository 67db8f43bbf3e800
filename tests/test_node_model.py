"""The node model bench.py prints beside its multi-GPU line (pico_amd/model.py,
VERDICT r3 item 6): its byte counts against the schedule facts the other CPU
tests establish (tests/test_direct_protocol.py's HBM table, the flat
phases' link loads of tests/test_schedule.py), its launch count against what
the direct transport's per-launch stamps counted on the GPU
(profiles/r4_dm_stamps_*), and its arithmetic."""
import pytest

import bench
from pico_amd import model as M

S3 = 67_108_864 * 4   # C3 bytes per rank


def test_link_bytes_of_the_c3_transports():
    # literal Bine: one peer per step, 2 (P-1)/P S over the busiest link in
    # total; the flat phases: (P-1)/P S spread over P-1 links per phase
    kw = dict(count=67_108_864, chunk_bytes=16 << 20)
    assert M.link_bytes("allreduce", "bine_bdw_remap", 8, transport="direct", **kw) == 1.75 * S3
    assert M.link_bytes("allreduce", "bine_bdw_remap", 8, transport="flatrs+flat", **kw) == 0.25 * S3
    assert M.link_bytes("allreduce", "bine_bdw_remap", 8, transport="flatrs+flat+dmt", **kw) == 0.25 * S3
    assert M.link_bytes("allreduce", "bine_bdw_remap", 4, transport="flatrs+flat", **kw) == 0.5 * S3


@pytest.mark.parametrize("P,fused,unfused", [(8, 6.375, 8.125), (4, 5.75, 7.25)])
def test_hbm_bytes_table(P, fused, unfused):
    # DESIGN.md's HBM table (also tests/test_direct_protocol.py at 1 MiB slots)
    kw = dict(count=67_108_864, chunk_bytes=16 << 20)
    assert M.hbm_bytes("allreduce", "bine_bdw_remap", P, transport="flatrs+flat+dmt", **kw) == fused * S3
    assert M.hbm_bytes("allreduce", "bine_bdw_remap", P, transport="flatrs+flat+dm", **kw) == unfused * S3
    # RCCL P2P moves bytes as the unfused direct transport does
    assert M.hbm_bytes("allreduce", "bine_bdw_remap", P, transport="flatrs+flat", **kw) == unfused * S3


def test_launch_count_matches_the_stamped_runs():
    # the per-exchange form (one_launch=False, BINE_DIRECT_FUSED_LARGE=0):
    # C3 at P = 2, 16 MiB chunks over flatrs+flat+dmt: 8 reduce-scatter
    # exchanges (each hosting the previous chunk's tree), the last tree by
    # itself, the 128 MiB allgather in 8 slot rounds (9 launches) = 18, the
    # launches per call tools/dm_stamps.py counted on the GPU; C4 33
    # (16 MiB slots, profiles/r4_dm_stamps_p2_solo.txt "base")
    s16 = dict(slot=16 << 20, one_launch=False)
    assert M.config_model("C3", 2, "flatrs+flat+dmt", **s16)["launches"] == 18
    assert M.config_model("C4", 2, "flatrs+flat+dmt", **s16)["launches"] == 33
    # P = 8: 2 exchanges of 16 MiB pieces, the last tree, the 32 MiB allgather
    # in 2 rounds (3 launches)
    assert M.config_model("C3", 8, "flatrs+flat+dmt", **s16)["launches"] == 6
    # the 64 MiB default slot (profiles/r4_dm_stamps_p2_sweep2.txt): the
    # allgather in 2 rounds at 16 MiB chunks (12), 4 + 1 + 1 at 64 MiB chunks
    # (6), C4 8 exchanges + the last tree (9); P = 8: the allgather in one
    o = dict(one_launch=False)
    assert M.config_model("C3", 2, "flatrs+flat+dmt", **o)["launches"] == 12
    assert M.config_model("C3", 2, "flatrs+flat+dmt", 64 << 20, **o)["launches"] == 6
    assert M.config_model("C4", 2, "flatrs+flat+dmt", 64 << 20, **o)["launches"] == 9
    assert M.config_model("C3", 8, "flatrs+flat+dmt", **o)["launches"] == 4


def test_one_launch_form():
    """round 5's default (bine_plan_dm_fused): a flat call whose chunks are
    slot-sized and fit one launch is ONE k_dm_fused launch -- C3 at P = 2 with
    64 MiB chunks (2 chunks + 2 allgather pieces per peer: tools/dm_stamps.py
    counted 1 launch per call, profiles/r5_dm_fused_p2.txt), C4 one launch per
    4 chunks (2 at P = 2, stamped), P = 4 / 8 one; 16 MiB chunks below the
    64 MiB slot keep the per-exchange launches.  The allgather's pushes come
    from registers: 0.5 S less HBM traffic at P = 2 than the per-exchange
    fused-tree form"""
    c64 = 64 << 20
    assert M.config_model("C3", 2, "flatrs+flat+dmt", c64)["launches"] == 1
    assert M.config_model("C4", 2, "flatrs+flat+dmt", c64)["launches"] == 2
    for P in (4, 8):
        assert M.config_model("C3", P, "flatrs+flat+dmt", c64)["launches"] == 1
        assert M.config_model("C4", P, "flatrs+flat+dmt", c64)["launches"] == 1
        assert M.config_model("C5", P, "flatrs+flat+dmt", c64)["launches"] == 1
    assert M.config_model("C3", 2, "flatrs+flat+dmt", 16 << 20)["launches"] == 12
    one = M.hbm_bytes("allreduce", "bine_bdw_remap", 2, count=67_108_864, chunk_bytes=c64)
    per = M.hbm_bytes("allreduce", "bine_bdw_remap", 2, count=67_108_864, chunk_bytes=c64, one_launch=False)
    assert (one, per) == (4.0 * S3, 4.5 * S3)
    assert M.hbm_bytes("allreduce", "bine_bdw_remap", 8, count=67_108_864, chunk_bytes=c64) == 5.5 * S3


def test_model_arithmetic():
    m = M.config_model("C3", 8, "flatrs+flat+dmt", link_gbs=100.0, hbm_rate_gbs=1000.0, t_boundary_us=10.0)
    t_link = 0.25 * S3 / 100e9 * 1e3
    t_hbm = 6.375 * S3 / 1000e9 * 1e3
    assert m["t_link_ms"] == pytest.approx(t_link, abs=1e-4)
    assert m["t_hbm_ms"] == pytest.approx(t_hbm, abs=1e-4)
    assert m["model_ms"] == pytest.approx(max(t_link, t_hbm) + m["launches"] * 10e-3, abs=1e-4)
    # one GPU shared by the ranks: every rank's bytes through one HBM, no link
    g = M.config_model("C3", 2, "flatrs+flat+dmt", one_gpu=True, hbm_rate_gbs=1000.0, t_boundary_us=0.0)
    assert g["t_link_ms"] == 0 and g["model_ms"] == pytest.approx(2 * g["hbm_bytes"] / 1e12 * 1e3, abs=1e-4)


def test_bench_maps_trial_names_to_the_model():
    a = bench.node_model("C3", 8, "flatrs+flat+dmt64x128", 16 << 20)
    b = bench.node_model("C3", 8, "flatrs+flat+dmt", 16 << 20)
    assert "error" not in a and a["model_ms"] == b["model_ms"]
    c = bench.node_model("C4", 8, "flatrs+flat+dm16", 64 << 20)
    assert "error" not in c and c["hbm_bytes"] == M.config_model("C4", 8, "flatrs+flat+dm", 64 << 20)["hbm_bytes"]


def test_c1_end_to_end_model():
    """C1 through the unchanged pico_core at P ranks with one
    GPU and one PCIe link each = the measured 1 MiB host round trip (P = 1,
    54 us with the kernels addressing the host buffers, round 6) + one
    k_dm_fused launch + 3 flag round trips + the busiest link's bytes.  Below
    the reference's own CPU libbine at P = 4 (215 us on the GPU box's cores)
    even with the device part at its one-GPU measured bound (49 us, ranks
    sharing one GPU); the one-GPU end-to-end runs (263 us at P = 4) put all
    four ranks' PCIe traffic on one link, which a node does not"""
    assert M.c1_e2e_us(1)["e2e_us"] == M.T_HOST_RT_US
    for P in (2, 4, 8):
        m = M.c1_e2e_us(P)
        lb = M.link_bytes("allreduce", "bine_bdw_remap", P, transport="flatrs+flat+dmt", count=262_144,
                          chunk_bytes=64 << 20)
        assert lb == 2 * (262_144 * 4) // P   # the flat phases: S / P on the busiest link, twice
        assert m["device_us"] == pytest.approx(M.T_BOUNDARY_US + 3 * M.T_FLAG_US + lb / (M.LINK_GBS * 1e3), abs=0.01)
        assert m["e2e_us"] < M.C1_REFERENCE_CPU_US[4]
    hi = M.T_HOST_RT_US + M.C1_ONE_GPU_DEV_US[4]
    assert hi < M.C1_REFERENCE_CPU_US[4]
