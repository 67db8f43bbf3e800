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


TYPES = {"0": "compute", "1": "sdma", "2": "sdma_xgmi"}


def _read(path):
    try:
        with open(path) as f:
            return f.read().strip()
    except OSError:
        return "?"


def queues(pid):
    """{(gpu_id, type): count} of one process's queues (None: not readable);
    pid in the host's numbering (KFD's sysfs is not namespaced)"""
    d = os.path.join(KFD, str(pid), "queues")
    try:
        out = {}
        for q in os.listdir(d):
            k = (_read(os.path.join(d, q, "gpuid")), TYPES.get(_read(os.path.join(d, q, "type")), "?"))
            out[k] = out.get(k, 0) + 1
        return out
    except OSError:
        return None


def gpus():
    """{gpu_id: pci location_id} of the GPUs in KFD's topology"""
    out = {}
    base = "/sys/class/kfd/kfd/topology/nodes"
    try:
        for n in os.listdir(base):
            g = _read(os.path.join(base, n, "gpu_id"))
            if g not in ("?", "0"):
                props = _read(os.path.join(base, n, "properties"))
                loc = [ln.split()[1] for ln in props.splitlines() if ln.startswith("location_id ")]
                out[g] = loc[0] if loc else "?"
    except OSError:
        pass
    return out


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
        for (g, t), v in q.items():
            tot[(g, t)] = tot.get((g, t), 0) + v
        try:
            with open(f"/proc/{p}/cmdline", "rb") as f:
                cmd = f.read().replace(b"\0", b" ").decode(errors="replace")[:80]
        except OSError:
            cmd = "?"
        lines.append(f"  pid {p}: {q}  {cmd}")
    tot = {f"gpu {g} {t}": v for (g, t), v in sorted(tot.items())}
    return (f"KFD queues, {len(lines)} processes (host pids, every GPU of the host), per GPU and type {tot}; "
            f"GPUs (gpu_id: pci location) {gpus()}\n" + "\n".join(lines))


def probe():
    import torch
    import pico_amd
    torch.cuda.init()
    torch.zeros(1, device="cuda").sum().item()
    pr = torch.cuda.get_device_properties(0)
    print("this process's GPU:", {k: getattr(pr, k, None) for k in ("name", "pci_bus_id", "pci_device_id",
                                                                       "pci_domain_id", "uuid")}, flush=True)
    print(summary(), flush=True)

    def mine():   # the host pid of this process is unknown (pid namespace): all processes' totals
        return summary().splitlines()[0]
    print("after torch init:", mine(), flush=True)
    ss = [torch.cuda.Stream() for _ in range(8)]
    for s in ss:
        with torch.cuda.stream(s):
            torch.ones(16, device="cuda").sum()
    torch.cuda.synchronize()
    print("after 8 normal streams ran a kernel:", mine(), flush=True)
    hs = [torch.cuda.Stream(priority=-1) for _ in range(8)]
    for s in hs:
        with torch.cuda.stream(s):
            torch.ones(16, device="cuda").sum()
    torch.cuda.synchronize()
    print("after 8 high-priority streams ran a kernel:", mine(), flush=True)
    for P in (2, 4, 8):
        cs = pico_amd.Comm.loopback(P, 0)
        n = 1 << 16
        sb = [torch.ones(n, device="cuda") for _ in range(P)]
        rb = [torch.empty(n, device="cuda") for _ in range(P)]
        pico_amd.loopback_allreduce(cs, "bine_bdw_remap", sb, rb, n, "float")
        torch.cuda.synchronize()
        print(f"after a loopback allreduce on {P} more comms:", mine(), flush=True)
    print(summary(), flush=True)


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "probe":
        sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        probe()
    else:
        print(summary())
