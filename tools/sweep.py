#!/usr/bin/env python3
"""GPU tuning sweep (not part of the product): render time of the octree
kernel per workload over launch-bounds variants (env RT_MIN_WAVES) and
culling slacks (rt_hip_set_cull_slack).

    python tools/sweep.py [--workloads c5,c3] [--minw 2,3,4,5] [--eps 256,32,8]
Writes gpurun_out/sweep.json; prints one line per config."""
import argparse
import json
import os
import sys
import tempfile
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "raytracing-gpu_amd"))
import numpy as np  # noqa: E402
import rtgpu  # noqa: E402
from bench import WORKLOADS, load_scene  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workloads", default="c5,c3")
    ap.add_argument("--minw", default="2,3,4,5")
    ap.add_argument("--eps", default="256,32,8")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--size-stop", default="", help="octree build knob list (env RT_OCT_SIZE_STOP)")
    ap.add_argument("--leaf", default="", help="octree leaf size list (env RT_OCT_LEAF)")
    a = ap.parse_args()
    out = []
    os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
    for wl_name in a.workloads.split(","):
        wl = WORKLOADS[wl_name]
        with tempfile.TemporaryDirectory() as td:
            s = load_scene(wl, td)
        f = s.frame()
        ref = None
        builds = [(ss, lf) for ss in (a.size_stop.split(",") if a.size_stop else [""])
                  for lf in (a.leaf.split(",") if a.leaf else [""])]
        for ss, lf in builds:
          for k, v in (("RT_OCT_SIZE_STOP", ss), ("RT_OCT_LEAF", lf)):
            if v:
                os.environ[k] = v
            else:
                os.environ.pop(k, None)
          t = time.perf_counter()
          ctx = rtgpu.Context(s, wl["accel"])
          info = ctx.info()
          print(json.dumps({"size_stop": ss, "leaf": lf, "build_s": time.perf_counter() - t,
                            "records": info["tri_refs"], "nodes": info["nodes"]}), flush=True)
          for eps in [float(x) for x in a.eps.split(",")]:
            ctx.set_cull_slack(eps)
            for mw in a.minw.split(","):
                os.environ["RT_MIN_WAVES"] = mw
                best = 1e9
                for _ in range(a.reps):
                    t = time.perf_counter()
                    img, st = ctx.render_image(f)
                    best = min(best, time.perf_counter() - t)
                if ref is None:
                    ref = img
                same = bool(np.array_equal(img.view(np.uint32), ref.view(np.uint32)))
                q = st["closest"] + st["shadow"]
                row = dict(workload=wl_name, size_stop=ss, leaf=lf, eps=eps, min_waves=int(mw),
                           ms=best * 1e3, mrays=q / best / 1e6, same_as_first=same)
                out.append(row)
                print(json.dumps(row), flush=True)
                with open(os.path.join(REPO, "gpurun_out", "sweep.json"), "w") as fo:
                    json.dump(out, fo, indent=1)
          ctx.close()


if __name__ == "__main__":
    main()
