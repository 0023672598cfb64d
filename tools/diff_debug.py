#!/usr/bin/env python3
"""GPU debugging aid (not part of the product): where do two octree renders
of the same frame differ, and which one matches the oracle there?

    python tools/diff_debug.py --grid 8 --eps-a 64 --eps-b 1e30 [--max 48]

eps 1e30 disables culling and pruning (every leaf is visited: brute force
through the tree).  Writes gpurun_out/diff_debug.json."""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "raytracing-gpu_amd"))
sys.path.insert(0, os.path.join(REPO, "oracle"))
import numpy as np  # noqa: E402
import rtgpu  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--grid", type=int, default=8)
    ap.add_argument("--tris", type=int, default=9766)
    ap.add_argument("--W", type=int, default=3840)
    ap.add_argument("--H", type=int, default=2160)
    ap.add_argument("--eps-a", default="64", help="comma list")
    ap.add_argument("--eps-b", type=float, default=1e30)
    ap.add_argument("--max", type=int, default=48)
    a = ap.parse_args()
    import oracle as orc
    s = rtgpu.Scene.synthetic(a.grid, a.grid, a.tris, seed=0x5EED, width=a.W, height=a.H)
    f = s.frame()
    import time
    ctx = rtgpu.Context(s, "octree")
    ctx.set_cull_slack(a.eps_b)
    t = time.perf_counter()
    ib, sb = ctx.render_image(f)
    print(f"reference eps {a.eps_b}: {time.perf_counter() - t:.3f} s", flush=True)
    sweep = []
    for e in [float(x) for x in a.eps_a.split(",")]:
        ctx.set_cull_slack(e)
        ia, sa = ctx.render_image(f)
        t = time.perf_counter()
        ia, sa = ctx.render_image(f)
        el = time.perf_counter() - t
        bad = np.argwhere((ia.view(np.uint32) != ib.view(np.uint32)).any(axis=2))
        sweep.append({"eps": e, "bad": int(len(bad)), "s": el})
        print(f"eps {e}: bad pixels {len(bad)}, {el*1e3:.1f} ms", flush=True)
    pix = bad[: a.max].astype(np.int32)
    out = {"grid": a.grid, "W": a.W, "H": a.H, "eps_ref": a.eps_b, "sweep": sweep, "pixels": []}
    if len(pix):
        vals, cnt = orc.render(s.ptr, a.W, a.H, pixels=pix, threads=16)
        for k, (r, c) in enumerate(pix):
            va, vb, vo = ia[r, c], ib[r, c], vals[k]
            row = {"r": int(r), "c": int(c), "a": va.tolist(), "b": vb.tolist(),
                   "oracle": vo.tolist(),
                   "a_ok": bool((va.view(np.uint32) == vo.view(np.uint32)).all()),
                   "b_ok": bool((vb.view(np.uint32) == vo.view(np.uint32)).all())}
            out["pixels"].append(row)
            print(json.dumps(row), flush=True)
    os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
    with open(os.path.join(REPO, "gpurun_out", f"diff_debug_g{a.grid}.json"), "w") as fo:
        json.dump(out, fo, indent=1)


if __name__ == "__main__":
    main()
