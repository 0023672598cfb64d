#!/usr/bin/env python3
"""Shadow queries of the headline frame, walk vs brute force (not part of
the product): renders C5 (octree_gpu), then rt_hip_verify_shadows shades
every stride-th hit record again through the shadow walk and by brute force
over all 10M triangles (cpu/hit.c:93-109) and compares each record's
per-light outcome.  Writes gpurun_out/c5_shadow_<tag>.json.

    python tools/c5_shadow.py --stride 16 [--policy 0]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "raytracing-gpu_amd"))
import rtgpu  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--grid", type=int, default=32)
    ap.add_argument("--W", type=int, default=3840)
    ap.add_argument("--H", type=int, default=2160)
    ap.add_argument("--stride", type=int, default=16)
    ap.add_argument("--policy", type=int, default=0)
    ap.add_argument("--tag", default="c5")
    ap.add_argument("--all", action="store_true", help="every record: --stride calls, one per offset")
    ap.add_argument("--exact", type=int, default=1,
                    help="proven light buffers (1, the library default) or slack-grown (0) (rt_hip_set_exact_shadows)")
    ap.add_argument("--probe", type=int, default=0,
                    help="also this many grazing triangles x 50 adversarial origins per light (tools/grazing.py), "
                         "light buffer vs brute force")
    a = ap.parse_args()
    s = rtgpu.Scene.synthetic(a.grid, a.grid, 9776, seed=0x5EED, width=a.W, height=a.H)
    ctx = rtgpu.Context(s, "octree_gpu")
    ctx.set_policy(a.policy)
    ctx.set_exact_shadows(bool(a.exact))
    info = ctx.info()
    img, st = ctx.render_image(s.frame())
    t = time.perf_counter()
    if a.all:
        v = {}
        for first in range(a.stride):
            w = ctx.verify_shadows(a.stride, first)
            for k, x in w.items():
                v[k] = v.get(k, 0) + x
            print(f"offset {first}/{a.stride}: {w}", flush=True)
    else:
        v = ctx.verify_shadows(a.stride)
    out = {"scene_triangles": s.triangle_count, "W": a.W, "H": a.H, "stride": a.stride,
           "policy": a.policy, "shadow_queries_in_frame": st["shadow"],
           "hit_records_in_frame": st["hit_records"], "shadow_global_prims": info["shadow_global"],
           "shadow_mu_max": info["shadow_mu_max"], "verify_seconds": time.perf_counter() - t,
           "exact_shadows": a.exact, "shadow_deferred": st.get("shadow_deferred", 0), "lightbuf": {k: info[k] for k in info if k.startswith("lightbuf")}, **v}
    if a.probe:
        sys.path.insert(0, os.path.join(REPO, "tools"))
        from grazing import grazing_origins
        tri = s.triangles_array()
        out["probe"] = []
        for li in range(s.s.light_count):
            L = s.s.lights[li]
            if int(L.type) not in (1, 2):
                continue
            lv = np.array([L.v.x, L.v.y, L.v.z], np.float64)
            o = grazing_origins(tri, int(L.type), lv, a.probe, 50)
            t = time.perf_counter()
            got = ctx.probe_shadows(li, o)
            ref = ctx.probe_shadows(li, o, brute=True)
            out["probe"].append({"light": li, "type": int(L.type), "origins": int(len(o)),
                                 "shadowed_frac": float(ref.mean()), "differ": int((got != ref).sum()),
                                 "buffer_lit_brute_shadowed": int((~got & ref).sum()),
                                 "seconds": time.perf_counter() - t})
    print(json.dumps(out), flush=True)
    os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
    with open(os.path.join(REPO, "gpurun_out", f"c5_shadow_{a.tag}.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
