"""Multi-process GPU checks run as a child process in its own process group:
on a time-out the whole group (the child and the rank processes it spawned)
is killed, so no orphaned rank keeps the GPU busy for the tests after it, and
the failure names the time-out instead of the run going silent.  Before the
kill the group gets SIGUSR1 (the rank processes of tools/staged_check.py dump
every thread's Python stack on it, faulthandler) and the failure carries the
box's process table, so a stall names where each rank waited."""
import os
import signal
import subprocess
import time


def run(cmd, env, timeout):
    p = subprocess.Popen(cmd, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True,
                         start_new_session=True)
    try:
        out, err = p.communicate(timeout=timeout)
    except subprocess.TimeoutExpired:
        try:
            ps = subprocess.run(["ps", "-eo", "pid,ppid,pgid,stat,etime,pcpu,rss,args", "--sort=pid"],
                                capture_output=True, text=True, timeout=20).stdout
        except Exception as e:  # noqa: BLE001 -- diagnostics only
            ps = f"(ps failed: {e})"
        try:
            os.killpg(p.pid, signal.SIGUSR1)
            time.sleep(3)
        except ProcessLookupError:
            pass
        os.killpg(p.pid, signal.SIGKILL)
        out, err = p.communicate()
        raise AssertionError(f"timed out after {timeout} s: {' '.join(cmd)}\n" + (out or "")[-3000:] +
                             (err or "")[-6000:] + "\nprocesses at the time-out:\n" + ps[-4000:])
    return subprocess.CompletedProcess(cmd, p.returncode, out, err)


def parent_state():
    """what this (pytest) process holds on the GPU and in page-locked host
    memory, printed before a multi-process check (shown with its failure)"""
    import sys
    torch = sys.modules.get("torch")
    if torch is None or not torch.cuda.is_initialized():
        print("parent: no GPU context", flush=True)
        return
    free, total = torch.cuda.mem_get_info()
    host = {}
    try:
        host = {k: v for k, v in torch.cuda.host_memory_stats().items() if "bytes" in k and "current" in k}
    except Exception:  # noqa: BLE001 -- diagnostics only
        pass
    print(f"parent: device free {free / 2**30:.1f} of {total / 2**30:.1f} GiB, torch reserved "
          f"{torch.cuda.memory_reserved() / 2**30:.1f} GiB, host pinned {host}", flush=True)
