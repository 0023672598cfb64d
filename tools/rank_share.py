#!/usr/bin/env python3
"""Per-rank cost of an N-way split on ONE GPU (not part of the product).

Renders rank r of an nranks-way split of the C5 frame (4x4-tile blocks dealt
round robin, csrc/rt_tiles.h; the work one GPU does in an N-GPU run, minus
the gather) and reports the HIP-event times of its candidate lists and its
three render kernels, for the strong-scaling estimate in DESIGN.md §7.

    python tools/rank_share.py --nranks 1 2 4 8 --steps 5
"""
import argparse
import ctypes as C
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "raytracing-gpu_amd"))
import rtgpu  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nranks", type=int, nargs="+", default=[1, 2, 4, 8])
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--all-ranks", action="store_true", help="every rank, not just the first and last")
    ap.add_argument("--out", default=os.path.join(REPO, "gpurun_out", "rank_share.json"))
    a = ap.parse_args()
    s = rtgpu.Scene.synthetic(32, 32, 9776, seed=0x5EED, width=3840, height=2160)
    f = s.frame()
    ctx = rtgpu.Context(s, "octree_gpu")
    L = rtgpu.lib()
    res = []
    for n in a.nranks:
        per = rtgpu.tile_buffer_floats(f.width, f.height, n)
        d = C.c_void_p()
        assert L.rt_hip_malloc(0, per * 4, C.byref(d)) == 0
        for rank in (range(n) if a.all_ranks else sorted({0, n - 1})):
            for _ in range(2):  # warm-up (the first may size the hit buffer: RT_EHITBUF)
                ctx.render(f, rank, n, d.value)
                try:
                    ctx.stats()
                    break
                except rtgpu.RtError as e:
                    if e.code != -10:
                        raise
            ctx.set_timing(True)
            t0 = time.perf_counter()
            for _ in range(a.steps):
                ctx.render(f, rank, n, d.value)
            ft = ctx.frame_times(a.steps)
            kt = ctx.kernel_times(a.steps)
            wall = (time.perf_counter() - t0) * 1e3 / a.steps
            st = ctx.stats()
            ctx.set_timing(False)
            lists = sum(x for x, _ in ft) / len(ft)
            kern = sum(y for _, y in ft) / len(ft)
            row = {"nranks": n, "rank": rank, "lists_ms": round(lists, 3), "render_ms": round(kern, 3),
                   "trace_ms": round(sum(x for x, _, _ in kt) / len(kt), 3),
                   "shade_ms": round(sum(y for _, y, _ in kt) / len(kt), 3),
                   "fold_ms": round(sum(z for _, _, z in kt) / len(kt), 3),
                   "frame_ms": round(lists + kern, 3), "wall_ms_per_frame": round(wall, 3), "cand_entries": st["cand_entries"],
                   "queries": st["closest"] + st["shadow"]}
            print(json.dumps(row), flush=True)
            res.append(row)
        L.rt_hip_free(d)
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    with open(a.out, "w") as fh:
        json.dump(res, fh, indent=1)


if __name__ == "__main__":
    main()
