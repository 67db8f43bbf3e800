#!/usr/bin/env python3
"""User-mode queues on the GPU, per process, from KFD's sysfs
(/sys/class/kfd/kfd/proc/<pid>/queues/<id>/type): how many compute / SDMA
queues every process holds.  Used by tests/_sub.py's diagnostics and by the
queue-count probe below.
usage: python tools/kfd_queues.py                  (every process)
       python tools/kfd_queues.py probe            (this process: queues after
                                                    creating streams / comms)"""
import os
import sys

KFD = "/sys/class/kfd/kfd/proc"


def queues(pid):
    """{type: count} of one process's queues (None: not readable)"""
    d = os.path.join(KFD, str(pid), "queues")
    try:
        out = {}
        for q in os.listdir(d):
            try:
                with open(os.path.join(d, q, "type")) as f:
                    t = f.read().strip()
            except OSError:
                t = "?"
            out[t] = out.get(t, 0) + 1
        return out
    except OSError:
        return None


def summary():
    """one line per process with queues, and the totals"""
    try:
        pids = sorted(int(p) for p in os.listdir(KFD) if p.isdigit())
    except OSError as e:
        return f"(no KFD sysfs: {e})"
    lines, tot = [], {}
    for p in pids:
        q = queues(p)
        if q is None:
            continue
        for k, v in q.items():
            tot[k] = tot.get(k, 0) + v
        try:
            with open(f"/proc/{p}/cmdline", "rb") as f:
                cmd = f.read().replace(b"\0", b" ").decode(errors="replace")[:80]
        except OSError:
            cmd = "?"
        lines.append(f"  pid {p}: {q}  {cmd}")
    return f"KFD queues, {len(lines)} processes, total {tot}\n" + "\n".join(lines)


def probe():
    import torch
    import pico_amd
    me = os.getpid()
    torch.cuda.init()
    torch.zeros(1, device="cuda").sum().item()
    print("after torch init:", queues(me), flush=True)
    ss = [torch.cuda.Stream() for _ in range(8)]
    for s in ss:
        with torch.cuda.stream(s):
            torch.ones(16, device="cuda").sum()
    torch.cuda.synchronize()
    print("after 8 normal streams ran a kernel:", queues(me), flush=True)
    hs = [torch.cuda.Stream(priority=-1) for _ in range(8)]
    for s in hs:
        with torch.cuda.stream(s):
            torch.ones(16, device="cuda").sum()
    torch.cuda.synchronize()
    print("after 8 high-priority streams ran a kernel:", queues(me), flush=True)
    for P in (2, 4, 8):
        cs = pico_amd.Comm.loopback(P, 0)
        n = 1 << 16
        sb = [torch.ones(n, device="cuda") for _ in range(P)]
        rb = [torch.empty(n, device="cuda") for _ in range(P)]
        pico_amd.loopback_allreduce(cs, "bine_bdw_remap", sb, rb, n, "float")
        torch.cuda.synchronize()
        print(f"after a loopback allreduce on {P} more comms:", queues(me), flush=True)
    print(summary(), flush=True)


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "probe":
        sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        probe()
    else:
        print(summary())
