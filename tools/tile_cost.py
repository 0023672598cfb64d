#!/usr/bin/env python3
"""Per-tile cost distribution of one frame (instrumented render kernel,
rt_hip_tile_cycles): how unevenly the 8x8 tiles cost, and the tail a
persistent-wave schedule can not hide.

    python tools/tile_cost.py --scene spheres --W 1920 --H 1080 [--accel octree]
    python tools/tile_cost.py --synthetic 32 --W 3840 --H 2160 [--nranks 8 --rank 0]
"""
import argparse
import ctypes as C
import gzip
import json
import os
import sys
import tempfile

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "raytracing-gpu_amd"))
import rtgpu  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scene", default=None)
    ap.add_argument("--synthetic", type=int, default=0)
    ap.add_argument("--W", type=int, default=1920)
    ap.add_argument("--H", type=int, default=1080)
    ap.add_argument("--accel", default="octree")
    ap.add_argument("--nranks", type=int, default=1)
    ap.add_argument("--rank", type=int, default=0)
    ap.add_argument("--out", default=None)
    ap.add_argument("--npy", default=None, help="also save per-tile clocks, (tx, ty) and entries (.npz)")
    a = ap.parse_args()
    if a.synthetic:
        s = rtgpu.Scene.synthetic(a.synthetic, a.synthetic, 9776, seed=0x5EED, width=a.W, height=a.H)
    else:
        src = os.path.join(REPO, "tests", "golden", "scenes", a.scene + ".svati.gz")
        with tempfile.TemporaryDirectory() as td:
            p = os.path.join(td, "s.svati")
            with gzip.open(src, "rb") as i, open(p, "wb") as o:
                o.write(i.read())
            s = rtgpu.Scene.load_svati(p)
        s.set_size(a.W, a.H)
    ctx = rtgpu.Context(s, a.accel)
    ctx.set_count_work(True)
    f = s.frame()
    L = rtgpu.lib()
    d = C.c_void_p()
    assert L.rt_hip_malloc(0, rtgpu.tile_buffer_floats(a.W, a.H, a.nranks) * 4, C.byref(d)) == 0
    for _ in range(2):  # the first render may size the hit buffer (RT_EHITBUF)
        ctx.render(f, a.rank, a.nranks, d.value)
        try:
            st = ctx.stats()
            break
        except rtgpu.RtError as e:
            if e.code != -10:
                raise
    nt = rtgpu.rank_tile_count(a.W, a.H, a.rank, a.nranks)  # rank-local tiles (csrc/rt_tiles.h order)
    txs, tys = rtgpu.tile_xy(np.arange(nt), a.rank, a.nranks, a.W, a.H)
    items = ctx.tile_cycles(4 * nt).astype(np.float64)  # item 4t + s = (tile t, sample s)
    c = items.reshape(-1, 4).sum(axis=1)
    # trace kernel phases (shadow queries run in the shade kernel, not per item)
    ph = {name: ctx.tile_phase_cycles(k, 4 * nt).astype(np.float64)
          for k, name in enumerate(("total", "camera_walk", "candidates", "secondary",
                                    "sec_lane_nodes_max", "sec_lane_tris_max")) if k}
    try:
        ent = ctx.cand_tile_entries(nt).astype(np.float64)
    except rtgpu.RtError:
        ent = None
    order = np.argsort(-c)
    tot = c.sum()
    res = {
        "nranks": a.nranks, "rank": a.rank,
        "tiles": int(len(c)), "total_clocks": tot, "mean": c.mean(), "max": c.max(),
        "p50": float(np.percentile(c, 50)), "p99": float(np.percentile(c, 99)),
        "max_over_mean": c.max() / c.mean(),
        "top1pct_share": float(c[order[: max(1, len(c) // 100)]].sum() / tot),
        # a persistent schedule of 4096 waves cannot finish before its most
        # expensive work item (one sample of a tile), nor before total / 4096
        "max_item": items.max(),
        "bound_tail_over_balanced": items.max() / (tot / 4096.0),
        # items per wave of the persistent grid (5 waves x 1024 SIMDs), and the
        # item-cost distribution in units of the mean item
        "items": int(len(items)), "mean_item": items.mean(),
        "items_over_mean": {str(k): int((items > k * items.mean()).sum()) for k in (2, 4, 8, 16)},
        "bound_tail_over_balanced_5120": items.max() / (items.sum() / 5120.0),
        "worst_tiles_rc": [[int(tys[i]) * 8, int(txs[i]) * 8] for i in order[:10]],
        "worst_items_cycles": [float(x) for x in np.sort(items)[::-1][:10]],
        # phase clocks of the 10 most expensive items and the mean item
        "worst_items_phases": [{k: float(ph[k][i]) for k in ph} for i in np.argsort(-items)[:10]],
        "mean_item_phases": {k: float(ph[k].mean()) for k in ph},
        # candidate entries of the worst tiles vs all tiles, and the correlation
        # of a tile's cost with its entry count
        "worst_tiles_entries": [float(ent[i]) for i in order[:10]] if ent is not None else None,
        "entries_mean_max": [float(ent.mean()), float(ent.max())] if ent is not None else None,
        "corr_cost_entries": float(np.corrcoef(c, ent)[0, 1]) if ent is not None else None,
        "stats": st,
    }
    print(json.dumps(res, default=float))
    if a.npy:
        np.savez_compressed(a.npy, cycles=c, tx=txs, ty=tys, items=items,
                            entries=ent if ent is not None else np.zeros(0))
    if a.out:
        with open(a.out, "w") as fh:
            json.dump(res, fh, default=float, indent=1)


if __name__ == "__main__":
    main()
