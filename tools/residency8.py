#!/usr/bin/env python3
"""Residency across PROCESSES: P processes on the one GPU,
each launching N / P workgroups of k_dm_fused's footprint
(tools/residency8.hip) that wait on ONE counter in device memory shared
between the processes (torch CUDA IPC), as the P ranks' k_dm_fused launches
wait on each other.  N completes iff all N are resident together; the
direct transport cuts each rank's launch to CUs x blocks per CU / P
(1,280 / 8 = 160 here).  One JSON line per N: how many workgroups timed out.
usage: python tools/residency8.py [P]"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "tools", "bin", "libresidency8.so")


def child(rank, P, per, n, shared, bar, q):
    import torch
    torch.cuda.set_device(0)
    L = ctypes.CDLL(LIB)
    L.residency8_launch.argtypes = [ctypes.c_void_p, ctypes.c_uint, ctypes.c_uint, ctypes.c_double, ctypes.c_void_p,
                                    ctypes.c_void_p]
    cnt, to = shared
    st = torch.cuda.Stream()
    bar.wait()   # every process ready: the launches go out together
    rc = L.residency8_launch(cnt.data_ptr(), n, per, 2.0, to.data_ptr(), st.cuda_stream)
    st.synchronize()
    q.put((rank, rc))


def main():
    import torch
    import torch.multiprocessing as mp
    P = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    ctx = mp.get_context("spawn")
    torch.cuda.set_device(0)
    props = torch.cuda.get_device_properties(0)
    nominal = props.multi_processor_count * 5
    for per in (nominal // P - 32, nominal // P - 8, nominal // P - 1, nominal // P, nominal // P + 1):
        n = per * P
        cnt = torch.zeros(1, dtype=torch.int32, device="cuda:0")
        to = torch.zeros(2, dtype=torch.int32, device="cuda:0")
        torch.cuda.synchronize()
        bar = ctx.Barrier(P)
        q = ctx.Queue()
        ps = [ctx.Process(target=child, args=(r, P, per, n, (cnt, to), bar, q)) for r in range(P)]
        for p in ps:
            p.start()
        for p in ps:
            p.join(120)
        rcs = sorted(q.get() for _ in ps if not q.empty())
        torch.cuda.synchronize()
        print(json.dumps({"processes": P, "workgroups_per_process": per, "workgroups": n, "nominal": nominal,
                          "arrived": int(cnt.item()), "timed_out_workgroups": int(to[0].item()),
                          "all_resident": int(to[0].item()) == 0, "launch_rcs": rcs}), flush=True)


if __name__ == "__main__":
    main()
