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
