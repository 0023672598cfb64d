#!/usr/bin/env python3
"""Render one workload a few times (for rocprofv3 kernel traces; not part of
the product).

    rocprofv3 --kernel-trace --stats -d gpurun_out/prof -- python3 tools/prof_render.py --grid 32
"""
import argparse
import ctypes as C
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "raytracing-gpu_amd"))
import rtgpu  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--grid", type=int, default=32)
    ap.add_argument("--tris", type=int, default=9776)
    ap.add_argument("--W", type=int, default=3840)
    ap.add_argument("--H", type=int, default=2160)
    ap.add_argument("--accel", default="octree_gpu")
    ap.add_argument("--n", type=int, default=3)
    ap.add_argument("--exact", type=int, default=1)
    ap.add_argument("--scale", type=float, default=1.0)
    ap.add_argument("--policy", type=int, default=0)
    ap.add_argument("--count", action="store_true", help="instrumented pass: print the work counters")
    a = ap.parse_args()
    s = rtgpu.Scene.synthetic(a.grid, a.grid, a.tris, seed=0x5EED, width=a.W, height=a.H)
    f = s.frame()
    ctx = rtgpu.Context(s, a.accel)
    ctx.set_exact_camera(bool(a.exact))
    ctx.set_camera_bound_scale(a.scale)
    ctx.set_policy(a.policy)
    if a.count:
        ctx.set_count_work(True)
    d = C.c_void_p()
    assert rtgpu.lib().rt_hip_malloc(0, rtgpu.tile_buffer_floats(a.W, a.H, 1) * 4, C.byref(d)) == 0
    for i in range(a.n):
        t = time.perf_counter()
        ctx.render(f, 0, 1, d.value)
        st = ctx.stats()
        print(f"render {i}: {(time.perf_counter() - t) * 1e3:.2f} ms, cand {st['cand_prims']} prims "
              f"{st['cand_entries']} entries", flush=True)
    if a.count:
        import json
        print(json.dumps(st), flush=True)


if __name__ == "__main__":
    main()
