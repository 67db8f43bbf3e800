"""Joining the rank processes of the multi-process probes: a rank that fails
leaves its peers blocked in a collective, so once any rank exits non-zero the
others are stopped (their exact Process objects) instead of waited for."""
import time


def join_ranks(ps, timeout_s):
    deadline = time.time() + timeout_s
    while any(p.is_alive() for p in ps) and time.time() < deadline:
        if any(p.exitcode not in (None, 0) for p in ps):
            print("a rank failed: exit codes", [p.exitcode for p in ps], "-- stopping the others", flush=True)
            break
        time.sleep(0.2)
    for p in ps:
        if p.is_alive():
            p.terminate()
        p.join(30)


def rank_device(rank):
    """the GPU a probe's rank uses: 0 (every rank on the box's one GPU, RCCL
    told the ranks are on different hosts so it moves bytes over sockets), or
    with BINE_RANK_DEVICES=1 on a multi-GPU node rank % the visible GPUs, RCCL
    left to find xGMI (tools/node_check.sh)"""
    import os
    if os.environ.get("BINE_RANK_DEVICES") == "1":
        import torch
        return rank % max(1, torch.cuda.device_count())
    os.environ["NCCL_HOSTID"] = f"bine-fake-host-{rank}"
    return 0
