"""Multi-process GPU checks run as a child process in its own process group:
on a time-out the whole group (the child and the rank processes it spawned)
is killed, so no orphaned rank keeps the GPU busy for the tests after it, and
the failure names the time-out instead of the run going silent."""
import os
import signal
import subprocess


def run(cmd, env, timeout):
    p = subprocess.Popen(cmd, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True,
                         start_new_session=True)
    try:
        out, err = p.communicate(timeout=timeout)
    except subprocess.TimeoutExpired:
        os.killpg(p.pid, signal.SIGKILL)
        out, err = p.communicate()
        raise AssertionError(f"timed out after {timeout} s: {' '.join(cmd)}\n" + (out or "")[-3000:] +
                             (err or "")[-2000:])
    return subprocess.CompletedProcess(cmd, p.returncode, out, err)
