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


def _self_cpu():
    t = os.times()
    return t.user + t.system


def _group_threads(pgid):
    """every thread of the process group: pid, tid, name, state, CPU seconds,
    kernel wait channel"""
    rows = []
    for pid in os.listdir("/proc"):
        if not pid.isdigit():
            continue
        try:
            with open(f"/proc/{pid}/stat") as f:
                st = f.read()
            if int(st[st.rindex(")") + 2:].split()[2]) != pgid:
                continue
            for tid in os.listdir(f"/proc/{pid}/task"):
                with open(f"/proc/{pid}/task/{tid}/stat") as f:
                    ts = f.read()
                name = ts[ts.index("(") + 1:ts.rindex(")")]
                fs = ts[ts.rindex(")") + 2:].split()
                try:
                    with open(f"/proc/{pid}/task/{tid}/wchan") as f:
                        wch = f.read().strip()
                except OSError:
                    wch = "?"
                cpu = (int(fs[11]) + int(fs[12])) / os.sysconf("SC_CLK_TCK")
                rows.append(f"{pid:>7} {tid:>7} {name:<16} {fs[0]} {cpu:8.1f}s {wch}")
        except (OSError, ValueError, IndexError):
            continue
    return "\n".join(rows)


def _sockets():
    """socket totals and TCP connections by state (/proc/net)"""
    out = []
    try:
        with open("/proc/net/sockstat") as f:
            out.append(f.read().strip())
        states = {}
        for fn in ("/proc/net/tcp", "/proc/net/tcp6"):
            with open(fn) as f:
                for ln in f.readlines()[1:]:
                    s = ln.split()[3]
                    states[s] = states.get(s, 0) + 1
        out.append("tcp states (hex, 01 established, 06 time_wait, 0A listen): " + str(sorted(states.items())))
    except OSError as e:
        out.append(f"(/proc/net: {e})")
    return "\n".join(out)


def _cpu_state():
    """the CPU budget this box gives us: the cgroup's throttling counters and
    the host's CPU pressure (when readable)"""
    st = {}
    try:
        with open("/proc/self/cgroup") as f:
            rel = f.read().strip().split("\n")[-1].split(":")[-1]
        for base in (f"/sys/fs/cgroup{rel}", "/sys/fs/cgroup"):
            if os.path.exists(f"{base}/cpu.stat"):
                with open(f"{base}/cpu.stat") as f:
                    st.update({k: int(v) for k, v in (ln.split() for ln in f if ln.strip())})
                with open(f"{base}/cpu.max") as f:
                    st["max"] = f.read().strip()
                break
    except (OSError, ValueError):
        pass
    try:
        with open("/proc/pressure/cpu") as f:
            st["psi_some_total_us"] = int(f.readline().split("total=")[1])
    except (OSError, IndexError, ValueError):
        pass
    return st


def cpu_delta(a, b, secs):
    """what changed between two _cpu_state() readings, per wall second"""
    out = {}
    for k in ("usage_usec", "throttled_usec", "nr_throttled", "psi_some_total_us"):
        if k in a and k in b:
            out[k + "_per_s"] = round((b[k] - a[k]) / max(secs, 1e-3), 1)
    if "max" in b:
        out["cpu.max"] = b["max"]
    return out


# HW queues per stream priority for each rank when several ranks share the
# test box's one GPU (HIP keeps a pool of GPU_MAX_HW_QUEUES queues per
# priority, plus one: tools/kfd_queues.py).  Past the GPU's hardware queue
# slots the scheduler time-slices the queues, and a rank whose queue is off
# the GPU stalls peers whose kernels spin waiting for it -- idle queues of
# another process are enough (tools/contention_probe.py,
# profiles/r4_queue_oversubscription.txt).  Measured in the
# suite (the test process at 2, tests/conftest.py): 4 ranks at HIP's 4 ran
# 3-10x slow and stalled the staged check; every rank count at 2 runs as fast
# as alone (the whole suite in 286 s, profiles/r4_gpu_suite.txt); 8 ranks at
# 1 took 4-7x longer (one queue serialises each rank's RCCL, copy and
# reduction launches).  The box exports GPU_MAX_HW_QUEUES=4, so the value is
# set, not defaulted (BINE_TEST_RANK_QUEUES overrides).  On a node every rank
# has a GPU of its own and HIP's default applies.
RANK_QUEUES = 2


def queues_per_rank(ranks):
    return RANK_QUEUES


def run_kw(cmd, env=None, capture_output=True, text=True, timeout=None, cwd=None, ranks=1, queues=None):
    """subprocess.run's keyword form of run() (its output always captured)"""
    assert capture_output and text
    return run(cmd, env, timeout, cwd=cwd, ranks=ranks, queues=queues)


def run(cmd, env, timeout, cwd=None, ranks=1, queues=None):
    """ranks > 1: the command starts that many GPU processes on the one GPU;
    each gets `queues` (default queues_per_rank()) HW queues per priority"""
    if ranks > 1:
        env = dict(os.environ if env is None else env)
        env["GPU_MAX_HW_QUEUES"] = str(queues) if queues else os.environ.get("BINE_TEST_RANK_QUEUES",
                                                                              str(queues_per_rank(ranks)))
    c0, w0 = _self_cpu(), time.time()
    s0 = _cpu_state()
    p = subprocess.Popen(cmd, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True,
                         start_new_session=True, cwd=cwd)
    try:
        out, err = p.communicate(timeout=timeout)
    except subprocess.TimeoutExpired:
        try:
            ps = subprocess.run(["ps", "-eo", "pid,ppid,pgid,stat,etime,pcpu,rss,args", "--sort=pid"],
                                capture_output=True, text=True, timeout=20).stdout
        except Exception as e:  # noqa: BLE001 -- diagnostics only
            ps = f"(ps failed: {e})"
        threads = _group_threads(p.pid) + "\n" + kfd_queues()
        sockets = _sockets()
        try:
            os.killpg(p.pid, signal.SIGUSR1)
            time.sleep(3)
        except ProcessLookupError:
            pass
        os.killpg(p.pid, signal.SIGKILL)
        out, err = p.communicate()
        raise AssertionError(f"timed out after {timeout} s: {' '.join(cmd)}\n" + (out or "")[-3000:] +
                             f"\nCPU budget meanwhile: {cpu_delta(s0, _cpu_state(), time.time() - w0)}\n" +
                             (err or "")[-6000:] + "\nprocesses at the time-out:\n" + ps[-4000:] +
                             "\nthreads of the group (pid tid name state cpu wchan):\n" + threads[-6000:] +
                             "\nsockets:\n" + sockets[-1500:] +
                             f"\nthis process meanwhile: {_self_cpu() - c0:.1f} s CPU in {time.time() - w0:.1f} s, "
                             f"{len(os.listdir('/proc/self/task'))} threads")
    print(f"[_sub] {os.path.basename(cmd[-3] if len(cmd) > 2 else cmd[0])} {time.time() - w0:.1f} s, CPU budget "
          f"meanwhile: {cpu_delta(s0, _cpu_state(), time.time() - w0)}", flush=True)
    return subprocess.CompletedProcess(cmd, p.returncode, out, err)


def kfd_queues():
    sys_path = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools")
    import sys
    if sys_path not in sys.path:
        sys.path.insert(0, sys_path)
    import kfd_queues as K
    return K.summary()


def parent_state():
    """what this (pytest) process holds on the GPU and in page-locked host
    memory, printed before a multi-process check (shown with its failure)"""
    import sys
    print("parent: " + _sockets().replace("\n", "; "), flush=True)
    print("parent: " + kfd_queues(), flush=True)
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
          f"{torch.cuda.memory_reserved() / 2**30:.1f} GiB, host pinned {host}, "
          f"{len(os.listdir('/proc/self/task'))} threads", flush=True)
