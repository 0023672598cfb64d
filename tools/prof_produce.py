#!/usr/bin/env python3
"""Time the triangle-parallel lists' produce step of an N-way split of the C5
frame, per producer (for rocprofv3 kernel traces; not part of the product).

    rocprofv3 --kernel-trace --stats -d gpurun_out/prod -- python3 tools/prof_produce.py --n 8

Prints the median host wall time of rt_hip_cand_produce per rank and, with
--trace <kernel_trace.csv> (a finished trace of this script), the per-kernel
GPU time of one produce and the part of the wall time no kernel covers.
"""
import argparse
import csv
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "raytracing-gpu_amd"))


def summarize(path, calls):
    """Per-kernel mean time per produce call from a rocprofv3 kernel trace."""
    per = {}
    rows = list(csv.DictReader(open(path)))
    for r in rows:
        k = r["Kernel_Name"].split("(")[0][:60]
        per[k] = per.get(k, 0.0) + (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
    return {k: round(v / calls, 4) for k, v in sorted(per.items(), key=lambda kv: -kv[1])}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=8)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--trace", help="kernel_trace.csv of an earlier run: per-kernel breakdown")
    ap.add_argument("--calls", type=int, default=0, help="produce calls in that trace")
    ap.add_argument("--consume", action="store_true", help="then rank 0's consume, --steps times")
    a = ap.parse_args()
    if a.trace:
        print(json.dumps(summarize(a.trace, a.calls), indent=1))
        return
    import rtgpu
    s = rtgpu.Scene.synthetic(32, 32, 9776, seed=0x5EED, width=3840, height=2160)
    f = s.frame()
    ctx = rtgpu.Context(s, "octree_gpu")
    for r in range(a.n):  # warm-up: buffers sized
        ctx.cand_produce(f, r, a.n)
    med = []
    for r in range(a.n):
        ts = []
        for _ in range(a.steps):
            t0 = time.perf_counter()
            ctx.cand_produce(f, r, a.n)
            ts.append((time.perf_counter() - t0) * 1e3)
        med.append(round(sorted(ts)[len(ts) // 2], 3))
    print(json.dumps({"n": a.n, "produce_ms": med, "max": max(med), "calls": a.n * (a.steps + 1)}), flush=True)
    if a.consume:  # rank 0's consume of what every producer routed to it, repeated
        import ctypes as C
        import numpy as np
        L = rtgpu.lib()
        blocks, g = [], 0
        for r in range(a.n):
            counts, ng = ctx.cand_produce(f, r, a.n)
            ptr, m = ctx.cand_send_buffer()
            host = np.empty((max(m, 1), 3), np.uint32)
            if m:
                assert L.rt_hip_memcpy_d2h(host.ctypes.data_as(C.c_void_p), C.c_void_p(ptr), m * 12) == 0
            blocks.append(host[:counts[0]])
            g += ng
        recv = np.ascontiguousarray(np.concatenate(blocks))
        dr = C.c_void_p()
        assert L.rt_hip_malloc(0, max(recv.nbytes, 16), C.byref(dr)) == 0
        assert L.rt_hip_memcpy_h2d(dr, recv.ctypes.data_as(C.c_void_p), recv.nbytes) == 0
        for _ in range(a.steps):  # (asynchronous: the kernel trace times them)
            ctx.cand_consume(f, 0, a.n, dr.value, len(recv), g)
        print(json.dumps({"consume_entries": int(len(recv)), "consume_calls": a.steps}), flush=True)


if __name__ == "__main__":
    main()
