#!/usr/bin/env python3
"""Host survey: which triangles' float Moller-Trumbore error region, for the
shadow rays of the scene's lights, can reach beyond the shadow walk's slack
(the per-light bound of DESIGN.md §2 "Exact shadow rays"; no GPU).

Shadow rays of a directional light all have the direction -l.v exactly
(cpu/light.c:53), so a triangle's grazing cosine is one number; those of a
point light all aim at the light (cpu/light.c:78: l.v - P), i.e. pass within
a few ulps of it, so the cosine is bounded below as for camera rays.  With
|S| = |o - v0| bounded over the scene box (a shadow ray starts on a surface),
tools/mt_bound.py's bound gives each triangle's expanded region T_D; the
triangle is safe when T_D lies within the walk's minimum slack of the
triangle.

    python tools/shadow_bound.py --synthetic 32 [--W 3840 --H 2160]
    python tools/shadow_bound.py --scene car-on-road
"""
import argparse
import gzip
import json
import os
import sys
import tempfile

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "raytracing-gpu_amd"))
import rtgpu  # noqa: E402

EPS = 2.0 ** -24
C_DOT, C_A = 8.6, 7.2
A_MIN = float(np.float32(1e-7))
DMAX = 1 + 4 * EPS


def lights_of(s):
    out = []
    for i in range(s.s.light_count):
        L = s.s.lights[i]
        out.append((int(L.type), np.array([L.v.x, L.v.y, L.v.z], np.float64)))
    return out


def survey(tri, lights, eps_ulps=64.0):
    v0 = tri[:, 0].astype(np.float64)
    e1 = (tri[:, 1] - tri[:, 0]).astype(np.float32).astype(np.float64)
    e2 = (tri[:, 2] - tri[:, 0]).astype(np.float32).astype(np.float64)
    allv = tri[:, :3].reshape(-1, 3).astype(np.float64)
    lo, hi = allv.min(0), allv.max(0)
    c = 0.5 * (lo + hi)
    R = 0.5 * (hi - lo).max()
    cmag = np.abs(c).max()
    eps_rel = eps_ulps * 5.9604645e-8
    omax = np.sqrt((np.maximum(np.abs(lo), np.abs(hi)) ** 2).sum())
    eps_min = (eps_rel * R + 2.384185791015625e-7 * (cmag + R) + 1e-6) * (1 - 1e-5)
    eps_avail = eps_min - 8 * EPS * (omax + 2 * (cmag + R))
    n = np.cross(e1, e2)
    nl = np.linalg.norm(n, axis=1)
    l1, l2 = np.linalg.norm(e1, axis=1), np.linalg.norm(e2, axis=1)
    # |S_i| <= max over the scene box of |o_i - v0_i| (a shadow origin lies on a surface)
    Smax = np.sqrt((np.maximum(np.abs(lo - v0), np.abs(hi - v0)) ** 2).sum(1)) * (1 + 1e-9)
    res = {"triangles": int(len(tri)), "eps_avail": eps_avail, "lights": []}
    for typ, lv in lights:
        if typ not in (1, 2):
            continue
        if typ == 1:
            D = -lv
            dl = np.linalg.norm(D)
            with np.errstate(all="ignore"):
                cl = np.nan_to_num(np.abs(n @ D) / (nl * dl))
        else:
            # rays (P, lv - P): lines through lv (within a few ulps); cosine >=
            # (distance of lv from the plane - slop) / (distance to the farthest vertex)
            with np.errstate(all="ignore"):
                dpl = np.nan_to_num(np.abs(((lv - v0) * n).sum(1)) / nl)
            vmax = np.max(np.linalg.norm(tri[:, :3].astype(np.float64) - lv, axis=2), axis=1)
            dline = 8 * EPS * (np.linalg.norm(lv) + omax + R)
            cl = np.maximum(0.0, (dpl - dline) / (vmax + dline))
            dl = 1.0  # the bound's du is scale-free in |d|
        e_a = C_A * EPS * l1 * l2 * DMAX
        a_lb = np.maximum(A_MIN, DMAX ** -2 * nl * cl - e_a)
        never = nl * DMAX + e_a < A_MIN
        rho = e_a / a_lb
        bad = rho >= 0.5
        e_sh = C_DOT * EPS * Smax * l2
        e_dq = C_DOT * EPS * Smax * l1
        with np.errstate(all="ignore"):
            du = e_sh / (a_lb * (1 - rho))
            dv = e_dq / (a_lb * (1 - rho))
            dw = (4 * EPS + (e_sh + e_dq) / a_lb + rho) / (1 - rho)
        # how far T_D's corners reach beyond the triangle
        reach = np.maximum.reduce([du * l1 + dv * l2, (dw + dv) * l1 + dv * l2, du * l1 + (dw + du) * l2])
        reach = np.where(never, 0.0, np.where(bad, np.inf, reach))
        safe = reach <= eps_avail
        q = np.quantile(reach[~safe & np.isfinite(reach)], [0.5, 0.9, 0.99]) if (~safe & np.isfinite(reach)).any() else []
        res["lights"].append({
            "type": "directional" if typ == 1 else "point", "v": lv.tolist(),
            "safe": int(safe.sum()), "fat": int((~safe & np.isfinite(reach)).sum()),
            "unbounded": int((~np.isfinite(reach)).sum()),
            "fat_reach_quantiles": [float(x) for x in q],
            "fat_reach_over_edge": [float(x) for x in np.quantile(
                (reach / np.maximum(l1, l2))[~safe & np.isfinite(reach)], [0.5, 0.9, 0.99, 0.999])]
            if (~safe & np.isfinite(reach)).any() else [],
            "fat_over_1pct_edge": int((~safe & (reach > 0.01 * np.maximum(l1, l2))).sum()),
            "min_cos_of_safe": float(cl[safe & ~never].min()) if (safe & ~never).any() else None})
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scene", default=None)
    ap.add_argument("--synthetic", type=int, default=0)
    ap.add_argument("--W", type=int, default=3840)
    ap.add_argument("--H", type=int, default=2160)
    ap.add_argument("--ulps", type=float, default=64.0)
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
    tri = s.triangles_array()
    print(json.dumps(survey(tri, lights_of(s), a.ulps), indent=1))


if __name__ == "__main__":
    main()
