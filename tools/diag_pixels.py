#!/usr/bin/env python3
"""Classify the differing pixels of tools/c5_exact.py (CPU, oracle side).

For every differing pixel, replay its oracle path (oracle/diag.c) and list
the queries whose deciding triangle the exact ray misses: `need` is how far
that triangle's box must grow for the exact ray to touch it, next to the
culling slack `eps` the kernel gives that ray (host/rt_cull.h rt_cull_eps).
A query with need > eps is one the octree walk may decide differently.

    python tools/diag_pixels.py gpurun_out/c5_exact_c5.json [--max 20]
"""
import argparse
import json
import os
import sys
from concurrent.futures import ThreadPoolExecutor

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "raytracing-gpu_amd"))
sys.path.insert(0, os.path.join(REPO, "oracle"))
import numpy as np  # noqa: E402
import oracle as orc  # noqa: E402
import rtgpu  # noqa: E402


def cull_eps(o, c, cmag, R, ulps=64.0):
    """host/rt_cull.h rt_cull_eps in float32, as the kernel computes it."""
    f = np.float32
    m = max(abs(f(o[0]) - f(c[0])), abs(f(o[1]) - f(c[1])), abs(f(o[2]) - f(c[2])))
    return float(f(ulps) * f(5.9604645e-8) * (f(m) + f(R)) + f(2.384185791015625e-7) * (f(cmag) + f(R))
                 + f(1e-6))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("json")
    ap.add_argument("--max", type=int, default=40)
    ap.add_argument("--threads", type=int, default=8)
    ap.add_argument("--key", default="differ", help="differ | differ_no_cand_px")
    a = ap.parse_args()
    res = json.load(open(a.json))
    if res.get("uv"):
        st, sl = (int(x) for x in res["uv"].split(","))
        s = rtgpu.Scene.synthetic_uv(res["grid"], res["grid"], st, sl, seed=0x5EED, width=res["W"],
                                     height=res["H"])
    else:
        s = rtgpu.Scene.synthetic(res["grid"], res["grid"], _tris_per(res), seed=0x5EED,
                                  width=res["W"], height=res["H"])
    tri = s.triangles_array()[:, :3]
    lo, hi = tri.reshape(-1, 3).min(axis=0), tri.reshape(-1, 3).max(axis=0)
    c = (np.float32(0.5) * (lo + hi)).astype(np.float32)
    R = float(np.max(np.float32(0.5) * (hi - lo)))
    cmag = float(np.max(np.abs(c)))
    pix = res[a.key][: a.max]

    def one(p):
        q, rgb = orc.diag_pixel(s.ptr, p["r"], p["c"])
        return p, q, rgb

    summary = {}
    out = []
    with ThreadPoolExecutor(a.threads) as ex:
        for p, q, rgb in ex.map(one, pix):
            flat_ok = bool((np.array(p["flat"], np.float32).view(np.uint32) ==
                            rgb.view(np.uint32)).all())
            bad = []
            for x in q:
                if x["obj"] < 0:
                    continue
                eps = cull_eps(x["o"], c, cmag, R)
                if x["need"] > eps:
                    x["eps"] = eps
                    # the error model of DESIGN.md: inplane <= kappa eps_f S shape / cos
                    x["kappa"] = x["inplane"] * x["cosn"] / (5.9604645e-8 * x["S"] * x["shape"])
                    bad.append(x)
                    summary[x["kind"]] = summary.get(x["kind"], 0) + 1
            row = {"r": p["r"], "c": p["c"], "flat_equals_oracle": flat_ok, "queries": len(q),
                   "culprits": [{k: x[k] for k in ("kind", "depth", "sample", "result", "obj", "tri",
                                                   "dist", "naccept", "u", "v", "cosn", "need",
                                                   "eps", "S", "inplane", "shape", "kappa", "kbary")} for x in bad]}
            out.append(row)
            print(json.dumps(row), flush=True)
    print("culprit queries by kind:", summary)
    with open(a.json.replace(".json", "_diag.json"), "w") as fo:
        json.dump({"pixels": out, "by_kind": summary}, fo, indent=1)


def _tris_per(res):
    # grid x grid spheres + 2 ground triangles
    return (res["tris"] - 2) // (res["grid"] * res["grid"])


if __name__ == "__main__":
    main()
