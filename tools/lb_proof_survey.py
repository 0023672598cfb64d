#!/usr/bin/env python3
"""Host survey for proven light buffers (no GPU; not part of the product).

For each triangle and light of a scene, the footprint a light buffer needs
so that every shadow ray the reference's float test (cpu/hit.c:15-33) can
accept finds the triangle in its cell (DESIGN.md §2 "Shadow rays"):

* directional light (rays (P, -l.v), cpu/light.c:53): the exact a = -d.n is
  one number per triangle; |a_f| >= 1e-7 is needed to accept, so the bound of
  tools/mt_bound.py with a_lb = max(1e-7, |a| - E_a) and |S| <= S_max gives the
  expanded triangle T_D, whose projection along the light is the footprint;
* point light (rays (P, l.v - P), cpu/light.c:78, lines through the light
  within dline): for rays at grazing cosine c >= c* the same bound with
  a_lb >= |d| (|n| c* - e_a) grows the triangle by R(c*) (the cone footprint);
  rays at c < c* can be accepted only from origins within H(c*) of the
  triangle's plane and nearly parallel to it, which needs the light within
  H(c*) of the plane -- else no band; otherwise a band of cells around the
  great circle of the plane through the light.

Prints the estimated entry counts of the proven footprints per light against
the current (slack-grown) ones.

    python tools/lb_proof_survey.py [--grid 32]
"""
import argparse
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "raytracing-gpu_amd"))
import rtgpu  # noqa: E402

EPS = 2.0 ** -24
C_DOT, C_A = 8.6, 7.2
A_MIN = float(np.float32(1e-7))
DMAX = 1 + 4 * EPS


def survey(tri, lights, nprim, ulps=64.0):
    v0 = tri[:, 0].astype(np.float64)
    e1 = (tri[:, 1] - tri[:, 0]).astype(np.float32).astype(np.float64)
    e2 = (tri[:, 2] - tri[:, 0]).astype(np.float32).astype(np.float64)
    allv = tri[:, :3].reshape(-1, 3).astype(np.float64)
    lo, hi = allv.min(0), allv.max(0)
    c = 0.5 * (lo + hi)
    R = 0.5 * (hi - lo).max()
    blo, bhi = c - R * 1.001 - 1e-3, c + R * 1.001 + 1e-3
    cmag = np.abs(c).max()
    eps_rel = ulps * 5.9604645e-8
    slack = (eps_rel * (2 * R * 1.001 + 1e-3) + 2.384185791015625e-7 * (cmag + R) + 1e-6) * 1.01
    n = np.cross(e1, e2)
    nl = np.linalg.norm(n, axis=1)
    l1, l2 = np.linalg.norm(e1, axis=1), np.linalg.norm(e2, axis=1)
    lmax, ls = np.maximum(l1, l2), l1 + l2
    Smax = np.sqrt((np.maximum(np.abs(blo - v0), np.abs(bhi - v0)) ** 2).sum(1)) * (1 + 1e-9)
    V = [v0, v0 + e1, v0 + e2]
    C = (V[0] + V[1] + V[2]) / 3
    rcirc = np.max([np.linalg.norm(x - C, axis=1) for x in V], axis=0)
    out = {"triangles": int(len(tri)), "slack": slack, "lights": []}
    for typ, lv in lights:
        if typ == 1:
            d = -lv
            dl = np.linalg.norm(d)
            A = np.abs(n @ d)                      # |a| exact, every ray of the light
            Ea = C_A * EPS * l1 * l2 * dl * DMAX
            never = A + Ea < A_MIN
            alb = np.maximum(A_MIN, A - Ea)
            rho = Ea / alb
            glob = (~never) & (rho >= 0.5)
            with np.errstate(all="ignore"):
                Esh = C_DOT * EPS * Smax * dl * l2
                Edq = C_DOT * EPS * Smax * dl * l1
                du = Esh / (alb * (1 - rho))
                dv = Edq / (alb * (1 - rho))
                dw = (4 * EPS + (Esh + Edq) / alb + rho) / (1 - rho)
            reach = np.maximum.reduce([du * l1 + dv * l2, (dw + dv) * l1 + dv * l2, du * l1 + (dw + du) * l2])
            ok = ~never & ~glob
            # footprint: projected T_D vs projected T grown by the slack (cells of side cs)
            cs = np.sqrt((2 * R) ** 2 * 1.0 / nprim)
            w = d / dl
            # projected area and perimeter of T (orthographic along w)
            pa = np.abs(n @ w) / 2
            per = ls + np.linalg.norm(e2 - e1, axis=1)
            cur = (pa + per * slack + np.pi * slack ** 2) / cs ** 2 + per / cs + 1
            grow = np.maximum(reach, 0)
            prov = (pa * (1 + du + dv + dw) ** 2 + per * (1 + du + dv + dw) * 1e-6 + per * grow + np.pi * grow ** 2) / cs ** 2 \
                + (per + 2 * np.pi * grow) / cs + 1
            out["lights"].append({
                "type": "directional", "never": int(never.sum()), "global": int(glob.sum()),
                "reach_quantiles": np.quantile(reach[ok], [0.5, 0.9, 0.99, 0.999, 1.0]).tolist(),
                "reach_over_slack_gt1": int((reach[ok] > slack).sum()),
                "cells_current_est": float(cur.sum()), "cells_proven_est": float(np.where(ok, prov, 0).sum())})
        else:
            D = lv - v0
            with np.errstate(all="ignore"):
                sL = np.abs((D * n).sum(1)) / nl
            Dmax = max(np.linalg.norm(np.array([[x, y, z] for x in (blo[0], bhi[0]) for y in (blo[1], bhi[1])
                                                for z in (blo[2], bhi[2])]) - lv, axis=1))
            dline = 2 * EPS * Dmax * np.sqrt(3)
            ea = C_A * EPS * l1 * l2 * DMAX           # E_a / |d|
            vdist = np.linalg.norm(C - lv, axis=1)
            ncube = int(np.ceil(np.sqrt(nprim / 6)))
            cell = 2.0 / ncube                         # radians, roughly (face centre)
            a_ = np.maximum(sL - dline, 0.0)
            b_ = vdist + rcirc + dline          # >= |L - v| for every vertex v, + dline

            def g(r, cst):
                """reach bound of rays crossing within r of T: their cosine >= c(r)"""
                cr = np.maximum(a_ / (b_ + r), cst)
                den = nl * cr - ea
                with np.errstate(all="ignore"):
                    rho = ea / den
                    kap = C_DOT * EPS / den
                    out = kap * ls * (lmax + ls) * Smax / (1 - rho) + (4 * EPS + rho) * lmax / (1 - rho)
                return np.where(den > 2.0001 * ea, out, np.inf)

            best = np.full(len(tri), np.inf)
            bestband = np.zeros(len(tri), bool)
            bestR = np.full(len(tri), np.inf)
            for cst in 10.0 ** np.arange(-6.5, -0.99, 0.5):
                # band needed when grazing rays (c < c*) can be accepted at all
                H = ls / (nl * (1 - cst)) * (nl * cst + ea + C_DOT * EPS * Smax * lmax + cst * Smax * lmax)
                band = sL <= H + Dmax * cst + dline
                # rays at c >= c*: smallest fixed point of r <= g(r) on [0, r_hi]
                r = np.zeros(len(tri))
                for _ in range(40):
                    r = g(r, 0.0) * 1.0001
                r_hi = a_ / cst - b_
                okfp = np.isfinite(r) & ((r_hi <= r) | (g(np.maximum(r_hi, r), 0.0) < np.maximum(r_hi, r)))
                # band triangles: rays at c >= c* bounded by g at c*
                rB = g(np.zeros(len(tri)), cst)
                Rc = np.where(band, np.maximum(np.where(okfp, r, rB), 0) if False else rB, np.where(okfp, r, np.inf))
                with np.errstate(all="ignore"):
                    rb = rcirc + Rc
                    th = np.arcsin(np.clip(rb / vdist, 0, 1)) + 4 * np.sqrt(3) * EPS * Dmax / np.maximum(vdist - rb, 1e-9)
                    cone = np.where(rb < 0.9 * vdist, np.pi * (th / cell) ** 2 + 2 * np.pi * th / cell + 1, np.inf)
                    bandcells = np.where(band, 4 * ncube * (2 * (cst + dline / 1.0) / cell + 2), 0)
                    tot = cone + bandcells
                better = tot < best
                best = np.where(better, tot, best)
                bestband = np.where(better, band, bestband)
                bestR = np.where(better, Rc, bestR)
            rb0 = rcirc + slack
            th0 = np.arcsin(np.clip(rb0 / vdist, 0, 1))
            cur = np.pi * (th0 / cell) ** 2 + 2 * np.pi * th0 / cell + 1
            fin = np.isfinite(best)
            out["lights"].append({
                "type": "point", "Dmax": Dmax, "n": ncube, "unbounded": int((~fin).sum()),
                "band": int(bestband[fin].sum()),
                "R_quantiles": np.quantile(bestR[fin], [0.5, 0.9, 0.99, 0.999, 1.0]).tolist(),
                "cells_current_est": float(cur.sum()), "cells_proven_est": float(best[fin].sum()),
                "cells_proven_band": float(best[fin & bestband].sum()),
                "sL_lt_1e-3": int((sL < 1e-3).sum()), "sL_lt_1e-2": int((sL < 1e-2).sum())})
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--grid", type=int, default=32)
    ap.add_argument("--tris", type=int, default=9776)
    a = ap.parse_args()
    s = rtgpu.Scene.synthetic(a.grid, a.grid, a.tris, seed=0x5EED, width=3840, height=2160)
    tri = s.triangles_array()[:, :3]
    lights = []
    for i in range(s.s.light_count):
        L = s.s.lights[i]
        if int(L.type) in (1, 2):
            lights.append((int(L.type), np.array([L.v.x, L.v.y, L.v.z], np.float64)))
    print(json.dumps(survey(tri, lights, len(tri)), indent=1))


if __name__ == "__main__":
    main()
