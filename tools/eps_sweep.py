#!/usr/bin/env python3
"""GPU experiment: octree culling slack vs exactness and speed.

For each scene, renders the brute-force (FLAT) image once, then the OCTREE
image at several slack values (rt_hip_set_cull_slack, in ulps of the
origin-to-scene distance), and reports pixels that differ from brute force
and the render time.  Writes gpurun_out/eps_sweep.json."""
import gzip
import json
import os
import sys
import tempfile
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "raytracing-gpu_amd"))
import rtgpu  # noqa: E402


def scene(name, W, H, td):
    if name.startswith("synthetic"):
        g = int(name.split(":")[1])
        return rtgpu.Scene.synthetic(g, g, 9766, seed=0x5EED, width=W, height=H)
    p = os.path.join(td, name + ".svati")
    with gzip.open(os.path.join(REPO, "tests", "golden", "scenes", name + ".svati.gz")) as i:
        open(p, "wb").write(i.read())
    s = rtgpu.Scene.load_svati(p)
    s.set_size(W, H)
    return s


def timed(ctx, f, reps=2):
    best = 1e9
    img = st = None
    for _ in range(reps):
        t = time.perf_counter()
        img, st = ctx.render_image(f)
        best = min(best, time.perf_counter() - t)
    return img, st, best


def main():
    cases = [("island_smooth", 1920, 1080), ("spheres", 1920, 1080), ("car-on-road", 3840, 2160),
             ("dark-night", 3840, 2160), ("susans_smooth", 1920, 1080),
             ("synthetic:8", 3840, 2160)]
    if os.environ.get("EPS_SWEEP_NO_SYNTH"):
        cases = cases[:-1]
    eps_list = [float(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "4,16,32,64,128,256").split(",")]
    out = []
    os.makedirs("gpurun_out", exist_ok=True)
    with tempfile.TemporaryDirectory() as td:
        for name, W, H in cases:
            s = scene(name, W, H, td)
            f = s.frame()
            flat = rtgpu.Context(s, "flat")
            ref, st_ref, t_ref = timed(flat, f, 1)
            flat.close()
            oc = rtgpu.Context(s, "octree")
            row = {"scene": name, "W": W, "H": H, "triangles": s.triangle_count,
                   "flat_s": t_ref, "queries": st_ref["closest"] + st_ref["shadow"], "octree": []}
            for e in eps_list:
                oc.set_cull_slack(e)
                img, st, t = timed(oc, f)
                bad = int((img.view(np.uint32) != ref.view(np.uint32)).any(axis=2).sum())
                row["octree"].append({"eps_ulps": e, "s": t, "bad_pixels": bad,
                                      "queries": st["closest"] + st["shadow"]})
                print(name, W, H, "eps", e, f"{t*1e3:.1f} ms", "bad", bad,
                      f"(flat {t_ref*1e3:.0f} ms)", flush=True)
            oc.close()
            out.append(row)
            with open("gpurun_out/eps_sweep.json", "w") as fo:
                json.dump(out, fo, indent=1)


if __name__ == "__main__":
    main()
