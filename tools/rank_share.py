#!/usr/bin/env python3
"""Per-rank cost of an N-way split on ONE GPU (not part of the product).

Renders rank r of an nranks-way split of the C5 frame (4x4-tile blocks, block
(bx, by) to rank (bx + by) mod N, csrc/rt_tiles.h; the work one GPU does in an N-GPU run, minus
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


def partition_cost(ctx, L, f, rank, n, d, steps):
    """Per-rank cost of the triangle-parallel lists for rank `rank` of n on
    one GPU: every producer's rt_hip_cand_produce (each rank runs its own in
    parallel: the slowest counts), then this rank's consume + render.  The
    all-to-all itself is not run here (one GPU): its bytes are reported."""
    import numpy as np
    prod_ms, parts = [], []
    for r in range(n):
        ts = []
        for _ in range(max(1, steps)):
            t0 = time.perf_counter()
            counts, ng = ctx.cand_produce(f, r, n)  # synchronises (the entry total)
            ts.append((time.perf_counter() - t0) * 1e3)
        ptr, m = ctx.cand_send_buffer()
        host = np.empty((max(m, 1), 3), np.uint32)
        if m:
            assert L.rt_hip_memcpy_d2h(host.ctypes.data_as(C.c_void_p), C.c_void_p(ptr), m * 12) == 0
        parts.append((host[:m], counts, ng))
        prod_ms.append(sorted(ts)[len(ts) // 2])
    blocks = []
    for host, counts, _ in parts:
        o = sum(counts[:rank])
        blocks.append(host[o:o + counts[rank]])
    recv = np.ascontiguousarray(np.concatenate(blocks))
    g = sum(p[2] for p in parts)
    sent = max(sum(c) - c[r] for r, (_, c, _) in enumerate(parts))
    dr = C.c_void_p()
    assert L.rt_hip_malloc(0, max(recv.nbytes, 16), C.byref(dr)) == 0
    assert L.rt_hip_memcpy_h2d(dr, recv.ctypes.data_as(C.c_void_p), recv.nbytes) == 0
    walls, frames = [], []
    ctx.set_timing(True)
    for _ in range(max(1, steps)):
        t0 = time.perf_counter()
        ctx.cand_consume(f, rank, n, dr.value, len(recv), g)
        ctx.render(f, rank, n, d.value)
        ctx.stats()  # waits for the render
        walls.append((time.perf_counter() - t0) * 1e3)
    ft = ctx.frame_times(max(1, steps))
    ctx.set_timing(False)
    L.rt_hip_free(dr)
    render = sum(y for _, y in ft) / len(ft)
    wall = sorted(walls)[len(walls) // 2]
    return {"partition": {"produce_ms_max": round(max(prod_ms), 3), "produce_ms": [round(x, 3) for x in prod_ms],
                          "consume_render_wall_ms": round(wall, 3), "render_ms": round(render, 3),
                          "consume_ms_est": round(wall - render, 3),
                          "received_entries": int(len(recv)), "received_bytes": int(recv.nbytes),
                          "max_sent_bytes": int(sent * 12),
                          "frame_ms_without_exchange": round(max(prod_ms) + wall, 3)}}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nranks", type=int, nargs="+", default=[1, 2, 4, 8])
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--all-ranks", action="store_true", help="every rank, not just the first and last")
    ap.add_argument("--reverse", action="store_true", help="measure the ranks in reverse order")
    ap.add_argument("--out", default=os.path.join(REPO, "gpurun_out", "rank_share.json"))
    ap.add_argument("--partition", action="store_true",
                    help="also the triangle-parallel lists (rt_hip_cand_produce / consume): each "
                         "producer timed, the all-to-all emulated on the host (its bytes reported)")
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
        ranks = list(range(n)) if a.all_ranks else sorted({0, n - 1})
        for rank in (ranks[::-1] if a.reverse else ranks):
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
            if a.partition and n > 1:
                row.update(partition_cost(ctx, L, f, rank, n, d, a.steps))
            print(json.dumps(row), flush=True)
            res.append(row)
        L.rt_hip_free(d)
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    with open(a.out, "w") as fh:
        json.dump(res, fh, indent=1)


if __name__ == "__main__":
    main()
