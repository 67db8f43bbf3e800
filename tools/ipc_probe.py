#!/usr/bin/env python3
"""Feasibility probe for a direct peer-access transport (a later round's
option beside RCCL P2P): can two processes sharing this box's GPU map each
other's device memory through HIP IPC handles (the mechanism a
one-process-per-GPU xGMI load/store transport would use)?

Process A allocates 64 MiB, fills it, exports hipIpcGetMemHandle; process B
opens it, copies it out, checks the bytes, writes a pattern back; A checks the
pattern.  Prints one JSON line.  usage: python tools/ipc_probe.py
"""
import ctypes
import json
import multiprocessing as mp
import sys

N = 64 << 20


def hip():
    h = ctypes.CDLL("libamdhip64.so")
    h.hipMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t]
    h.hipMemset.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t]
    h.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    h.hipIpcGetMemHandle.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    h.hipIpcOpenMemHandle.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_char * 64, ctypes.c_uint]
    h.hipIpcCloseMemHandle.argtypes = [ctypes.c_void_p]
    h.hipDeviceSynchronize.argtypes = []
    return h


def owner(q_out, q_in):
    h = hip()
    p = ctypes.c_void_p()
    assert h.hipMalloc(ctypes.byref(p), N) == 0
    assert h.hipMemset(p, 0x5A, N) == 0
    assert h.hipDeviceSynchronize() == 0
    hd = (ctypes.c_char * 64)()
    rc = h.hipIpcGetMemHandle(hd, p)
    q_out.put((rc, bytes(hd)))
    verdict = q_in.get(timeout=120)
    host = (ctypes.c_ubyte * N)()
    h.hipMemcpy(host, p, N, 2)  # D2H
    q_out.put(("owner_sees_pattern", all(host[i] == 0xA5 for i in range(0, N, 4099)), verdict))


def peer(q_in, q_out):
    h = hip()
    rc, hd = q_in.get(timeout=120)
    res = {"get_handle_rc": rc}
    if rc != 0:
        q_out.put(res)
        return
    p = ctypes.c_void_p()
    buf = (ctypes.c_char * 64).from_buffer_copy(hd)
    res["open_rc"] = h.hipIpcOpenMemHandle(ctypes.byref(p), buf, 1)  # hipIpcMemLazyEnablePeerAccess
    if res["open_rc"] == 0:
        host = (ctypes.c_ubyte * N)()
        res["read_rc"] = h.hipMemcpy(host, p, N, 2)
        res["peer_reads_owner_bytes"] = all(host[i] == 0x5A for i in range(0, N, 4099))
        res["write_rc"] = h.hipMemset(p, 0xA5, N)
        h.hipDeviceSynchronize()
        res["close_rc"] = h.hipIpcCloseMemHandle(p)
    q_out.put(res)


if __name__ == "__main__":
    ctx = mp.get_context("spawn")
    a2b, b2a = ctx.Queue(), ctx.Queue()
    pa = ctx.Process(target=owner, args=(a2b, b2a))
    pb = ctx.Process(target=peer, args=(a2b, b2a))
    pa.start()
    pb.start()
    pb.join(180)
    pa.join(180)
    out = {}
    while not a2b.empty():
        x = a2b.get()
        if isinstance(x, tuple) and x and x[0] == "owner_sees_pattern":
            out["owner_sees_peer_writes"] = x[1]
            out.update(x[2])
    out["exitcodes"] = [pa.exitcode, pb.exitcode]
    print(json.dumps(out), flush=True)
    sys.exit(0)
