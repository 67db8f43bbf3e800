#!/usr/bin/env python3
"""What slows the multi-process staged check down inside the GPU suite
(tests/test_gpu_rccl.py::test_staged_host_buffers_4_ranks: 10 s by itself,
>170 s after the suite's in-process tests, every case ~10x slower, the ranks
finally stuck in torch.cuda.synchronize with 190 % CPU each): the check run
beside a "holder" process that keeps one kind of state the suite's pytest
process may hold, one holder at a time:
  none      no holder
  ctx       a GPU context with 8 idle streams
  dev:G     G GiB of device memory (torch caching allocator)
  pin:G     G GiB of page-locked host memory (torch's host caching allocator)
  reg:G     G GiB of malloc'd host memory registered with hipHostRegister
  q:N       N streams that have each run a kernel (HW queues created; the
            holder runs with GPU_MAX_HW_QUEUES=N)
A holder spec may end in /VAR=val,VAR=val: environment of the check's ranks
(e.g. none/GPU_MAX_HW_QUEUES=8).
usage: python tools/contention_probe.py HOLDER [HOLDER ...]   (one JSON line each)
"""
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

HOLD = r"""
import sys, time, ctypes, torch
kind, g = sys.argv[1], float(sys.argv[2])
n = int(g * (1 << 30))
keep = []
torch.cuda.init()
free0, tot = torch.cuda.mem_get_info()
if kind == "ctx":
    keep = [torch.cuda.Stream() for _ in range(8)]
    torch.zeros(1, device="cuda").sum().item()
elif kind == "dev":
    step = 1 << 30
    for _ in range(max(1, n // step)):
        keep.append(torch.empty(step, dtype=torch.uint8, device="cuda"))
    torch.cuda.synchronize()
elif kind == "q":
    keep = [torch.cuda.Stream() for _ in range(int(g))]
    for s in keep:
        with torch.cuda.stream(s):
            torch.ones(1024, device="cuda").sum()
    torch.cuda.synchronize()
elif kind == "pin":
    step = 256 << 20
    for _ in range(max(1, n // step)):
        t = torch.empty(step, dtype=torch.uint8).pin_memory()
        keep.append(t)
elif kind == "reg":
    hip = ctypes.CDLL("libamdhip64.so")
    step = 256 << 20
    for _ in range(max(1, n // step)):
        b = ctypes.create_string_buffer(step)
        rc = hip.hipHostRegister(ctypes.c_void_p(ctypes.addressof(b)), ctypes.c_size_t(step), ctypes.c_uint(0))
        assert rc == 0, rc
        keep.append(b)
free1, _ = torch.cuda.mem_get_info()
print(f"HOLDING {kind} {g} GiB: device free {free0 / 2**30:.1f} -> {free1 / 2**30:.1f} of {tot / 2**30:.1f} GiB",
      flush=True)
time.sleep(600)
"""


def probe(spec):
    hspec, _, renv = spec.partition("/")
    kind, _, g = hspec.partition(":")
    holder = None
    line = ""
    if kind != "none":
        henv = dict(os.environ, GPU_MAX_HW_QUEUES=g) if kind == "q" else None
        holder = subprocess.Popen([sys.executable, "-c", HOLD, kind, g or "0"], stdout=subprocess.PIPE, text=True,
                                  start_new_session=True, env=henv)
        line = holder.stdout.readline().strip()
    t0 = time.time()
    env = dict(os.environ, PYTHONPATH=ROOT, BINE_SYNC_TIMEOUT_S="60")
    env.update(dict(x.split("=", 1) for x in renv.split(",") if x))
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import _sub
    try:
        r = _sub.run([sys.executable, "-u", os.path.join(ROOT, "tools", "staged_check.py"), "4", "1"], env=env,
                     timeout=90)
        rc, tail = r.returncode, r.stdout.splitlines()[-1:]
    except AssertionError as e:
        txt = str(e)
        rc, tail = "timeout", [ln for ln in txt.splitlines() if "start" in ln or "ok" in ln][-8:] + \
            txt[txt.find("threads of the group"):].splitlines()[:60]
    dt = time.time() - t0
    if holder:
        os.killpg(holder.pid, 9)
        holder.wait()
    print(json.dumps({"holder": spec, "holder_says": line, "rc": rc, "seconds": round(dt, 1), "tail": tail}),
          flush=True)
    return rc == 0


if __name__ == "__main__":
    ok = True
    for s in sys.argv[1:]:
        ok = probe(s) and ok
    sys.exit(0 if ok else 1)
