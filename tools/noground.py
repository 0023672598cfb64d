#!/usr/bin/env python3
"""C5 without its ground quad (an experiment, not part of the product).

Round 2 asked whether the ground quad's clipped references make the most
expensive work items of the C5 frame expensive; its script advanced the
library-owned scene's `objects` pointer past the ground object, and
rt_scene_free then freed an interior pointer ("double free or corruption
(out)" at exit, profiles/r02n_c5/no_ground_experiment.log).  The supported
way is to empty the object in place: objects[0].triangle_count = 0 (the
ground is object 0 of rt_scene_synthetic, host/synth.c), which the library
frees normally.  Prints the worst work items of the instrumented trace
kernel and the frame time, with and without the ground.

    python tools/noground.py [--W 3840 --H 2160]
"""
import argparse
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "raytracing-gpu_amd"))
import rtgpu  # noqa: E402


def run(scene, W, H, tag):
    ctx = rtgpu.Context(scene, "octree_gpu")
    f = scene.frame()
    ctx.render_image(f)  # warm-up (and the hit buffers)
    ctx.set_timing(True)
    for _ in range(3):
        ctx.render_image(f)
    ft = ctx.frame_times(3)
    kt = ctx.kernel_times(3)
    ctx.set_timing(False)
    ctx.set_count_work(True)
    ctx.render_image(f)
    nt = rtgpu.rank_tile_count(W, H, 0, 1)
    items = ctx.tile_cycles(4 * nt).astype(np.float64)
    txs, tys = rtgpu.tile_xy(np.arange(nt), 0, 1, W, H)
    order = np.argsort(-items)[:5]
    res = {"tag": tag, "triangles": scene.triangle_count, "info": ctx.info(),
           "lists_ms": min(a for a, _ in ft), "render_ms": min(b for _, b in ft),
           "kernels_ms": [list(k) for k in kt],
           "max_item": float(items.max()), "mean_item": float(items.mean()),
           "worst_items": [{"row": int(tys[i // 4]) * 8, "col": int(txs[i // 4]) * 8,
                            "sample": int(i % 4), "clocks": float(items[i])} for i in order]}
    ctx.close()
    print(json.dumps(res, default=float), flush=True)
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--W", type=int, default=3840)
    ap.add_argument("--H", type=int, default=2160)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    s = rtgpu.Scene.synthetic(32, 32, 9776, seed=0x5EED, width=a.W, height=a.H)
    out = [run(s, a.W, a.H, "with ground")]
    ground = s.s.objects[0]
    assert ground.triangle_count == 2, "object 0 of the synthetic scene is the ground quad"
    ground.triangle_count = 0  # emptied in place: objects[] and its allocations stay the library's
    out.append(run(s, a.W, a.H, "without ground"))
    s.close()  # rt_scene_free: every triangles[] block and objects[] as allocated
    if a.out:
        with open(a.out, "w") as fh:
            json.dump(out, fh, indent=1, default=float)


if __name__ == "__main__":
    main()
