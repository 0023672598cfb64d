#!/usr/bin/env python3
"""Parity measurement on the headline scene (not part of the product).

Renders the synthetic scene with the octree (device-built by default) over
the whole frame and with brute force (RT_ACCEL_FLAT, the reference's own
collide/collide_dist, cpu/hit.c:72-109) over a tile subsample -- the tiles of
ranks `--ranks` of an `--nranks`-way interleaved split, i.e. every nranks-th
8x8 tile -- and compares them bit for bit.  Writes
gpurun_out/c5_exact_<tag>.json with every differing pixel (both values), the
octree frame time and the optional culling-slack sweep.

    python tools/c5_exact.py --grid 32 --tris 9776 --W 3840 --H 2160 --nranks 64 --ranks 0
"""
import argparse
import ctypes as C
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "raytracing-gpu_amd"))
import numpy as np  # noqa: E402
import rtgpu  # noqa: E402


def log(*a):
    print(*a, flush=True)


def render_rank(ctx, f, rank, nranks):
    L = rtgpu.lib()
    per = rtgpu.tile_buffer_floats(f.width, f.height, nranks)
    d = C.c_void_p()
    assert L.rt_hip_malloc(0, per * 4, C.byref(d)) == 0
    ctx.render(f, rank, nranks, d.value)
    st = ctx.stats()
    out = np.empty(per, np.float32)
    assert L.rt_hip_memcpy_d2h(out.ctypes.data_as(C.c_void_p), d, out.nbytes) == 0
    L.rt_hip_free(d)
    return out.reshape(-1, 64, 3), st


def tile_pixels(f, rank, nranks):
    """(tiles, 64, 2) PPM (row, col) of the rank's tile buffer slots (-1 = pad)."""
    return rtgpu.tile_pixels(f.width, f.height, rank, nranks)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--grid", type=int, default=32)
    ap.add_argument("--tris", type=int, default=9776)
    ap.add_argument("--W", type=int, default=3840)
    ap.add_argument("--H", type=int, default=2160)
    ap.add_argument("--accel", default="octree_gpu")
    ap.add_argument("--nranks", type=int, default=64)
    ap.add_argument("--ranks", default="0")
    ap.add_argument("--slacks", default="", help="extra culling slacks (ulps) to compare")
    ap.add_argument("--tag", default="c5")
    ap.add_argument("--uv", default="", help="explicit stacks,slices (round 1's C5: 258,19)")
    ap.add_argument("--scale", type=float, default=None, help="camera bound scale (default: library)")
    a = ap.parse_args()
    if a.uv:
        st, sl = (int(x) for x in a.uv.split(","))
        s = rtgpu.Scene.synthetic_uv(a.grid, a.grid, st, sl, seed=0x5EED, width=a.W, height=a.H)
    else:
        s = rtgpu.Scene.synthetic(a.grid, a.grid, a.tris, seed=0x5EED, width=a.W, height=a.H)
    f = s.frame()
    t = time.perf_counter()
    ctx = rtgpu.Context(s, a.accel)
    if a.scale is not None:
        ctx.set_camera_bound_scale(a.scale)
    log(f"scene {s.triangle_count} tris, {a.accel} ctx {time.perf_counter() - t:.2f}s")
    img, st = ctx.render_image(f)
    L = rtgpu.lib()
    times = []
    for _ in range(3):
        t = time.perf_counter()
        ctx.render(f, 0, 1, _tiles_buf(f))
        ctx.stats()
        times.append(time.perf_counter() - t)
    log(f"{a.accel} full frame: {min(times) * 1e3:.2f} ms (best of 3), {st['closest']} closest "
        f"{st['shadow']} shadow, candidates: {st['cand_prims']} prims {st['cand_entries']} entries "
        f"{st['cand_global']} global")
    # the same walk without the camera candidate lists (A/B)
    ctx.set_exact_camera(False)
    img_nc, _ = ctx.render_image(f)
    tn = []
    for _ in range(3):
        t = time.perf_counter()
        ctx.render(f, 0, 1, _tiles_buf(f))
        ctx.stats()
        tn.append(time.perf_counter() - t)
    ctx.set_exact_camera(True)
    log(f"{a.accel} without candidate lists: {min(tn) * 1e3:.2f} ms")
    ranks = []
    for x in a.ranks.split(","):  # "0,5,9" or ranges "0-127"
        if "-" in x:
            lo, hi = (int(y) for y in x.split("-"))
            ranks.extend(range(lo, hi + 1))
        elif x != "":
            ranks.append(int(x))
    flat = rtgpu.Context(s, "flat")
    out = {"grid": a.grid, "tris": s.triangle_count, "W": a.W, "H": a.H, "accel": a.accel,
           "nranks": a.nranks, "ranks": ranks, "octree_ms": min(times) * 1e3, "octree_stats": st,
           "uv": a.uv, "octree_ms_no_cand": min(tn) * 1e3, "differ_no_cand": 0,
           "pixels_compared": 0, "differ": [], "differ_no_cand_px": [], "slack_sweep": []}
    imgs = {}
    for sl in [float(x) for x in a.slacks.split(",") if x]:
        ctx.set_cull_slack(sl)
        im, _ = ctx.render_image(f)
        t = time.perf_counter()
        ctx.render(f, 0, 1, _tiles_buf(f))
        ctx.stats()
        imgs[sl] = (im, time.perf_counter() - t)
    for r in ranks:
        t = time.perf_counter()
        tf, stf = render_rank(flat, f, r, a.nranks)
        el = time.perf_counter() - t
        pix = tile_pixels(f, r, a.nranks)
        tf = tf[: len(pix)]
        ok = pix[..., 0] >= 0
        pr, pc = pix[..., 0][ok], pix[..., 1][ok]
        vf = tf[ok]
        vo = img[pr, pc]
        d = (vf.view(np.uint32) != vo.view(np.uint32)).any(axis=1)
        out["pixels_compared"] += int(ok.sum())
        dn = (vf.view(np.uint32) != img_nc[pr, pc].view(np.uint32)).any(axis=1)
        out["differ_no_cand"] += int(dn.sum())
        for k in np.flatnonzero(dn):
            out["differ_no_cand_px"].append({"r": int(pr[k]), "c": int(pc[k]), "flat": vf[k].tolist(),
                                             "octree": img_nc[pr[k], pc[k]].tolist()})
        log(f"rank {r}/{a.nranks}: flat {el:.1f}s, {stf['closest']} closest {stf['shadow']} shadow, "
            f"{int(ok.sum())} px, {int(d.sum())} differ ({int(dn.sum())} without candidate lists)")
        for k in np.flatnonzero(d):
            out["differ"].append({"r": int(pr[k]), "c": int(pc[k]), "flat": vf[k].tolist(),
                                  "octree": vo[k].tolist()})
        if r % 8 == 7 or r == ranks[-1]:  # partial results survive a cut-off run
            _dump(out, a.tag)
        for sl, (im, el2) in imgs.items():
            ds = (vf.view(np.uint32) != im[pr, pc].view(np.uint32)).any(axis=1)
            out["slack_sweep"].append({"rank": r, "slack": sl, "ms": el2 * 1e3, "differ": int(ds.sum())})
            log(f"  slack {sl}: {el2 * 1e3:.1f} ms, {int(ds.sum())} differ")
    _dump(out, a.tag)
    log(json.dumps({k: v for k, v in out.items() if k not in ("differ", "octree_stats")}))


def _dump(out, tag):
    out["differ_count"] = len(out["differ"])
    os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
    with open(os.path.join(REPO, "gpurun_out", f"c5_exact_{tag}.json"), "w") as fo:
        json.dump(out, fo, indent=1)


_buf = {}


def _tiles_buf(f):
    key = (f.width, f.height)
    if key not in _buf:
        d = C.c_void_p()
        assert rtgpu.lib().rt_hip_malloc(0, rtgpu.tile_buffer_floats(f.width, f.height, 1) * 4,
                                         C.byref(d)) == 0
        _buf[key] = d.value
    return _buf[key]


if __name__ == "__main__":
    main()
