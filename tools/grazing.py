"""Adversarial shadow-ray origins (tests and tools; not part of the product)."""
import numpy as np


def grazing_origins(tri, light_type, lv, n_tri, per_tri, seed=1):
    """Adversarial shadow-ray origins for light (light_type, lv): for the n_tri
    triangles whose planes the light's rays graze most (directional: the
    smallest |n.d|; point: the light closest to the plane relative to its
    distance), points X around each triangle (barycentrics in [-0.5, 1.5])
    and origins on the shadow ray's line through X, on the far side from the
    light -- so every ray crosses the plane right at the triangle, at the
    most grazing angles the scene offers.  Kept inside the scene cube (the
    origin box the proof assumes)."""
    rng = np.random.default_rng(seed)
    v = tri[:, :3].astype(np.float64)
    v0, e1, e2 = v[:, 0], v[:, 1] - v[:, 0], v[:, 2] - v[:, 0]
    nrm = np.cross(e1, e2)
    nl = np.linalg.norm(nrm, axis=1)
    ok = nl > 0
    if light_type == 1:
        d = -lv / np.linalg.norm(lv)
        g = np.where(ok, np.abs(nrm @ d) / np.maximum(nl, 1e-300), np.inf)
    else:
        C = v.mean(axis=1)
        g = np.where(ok, np.abs(((lv - v0) * nrm).sum(1)) / np.maximum(nl, 1e-300)
                     / np.linalg.norm(C - lv, axis=1), np.inf)
    pick = np.argsort(g)[:n_tri]
    a = rng.uniform(-0.5, 1.5, (n_tri, per_tri, 1))
    b = rng.uniform(-0.5, 1.5, (n_tri, per_tri, 1))
    X = v0[pick][:, None] + a * e1[pick][:, None] + b * e2[pick][:, None]
    if light_type == 1:
        lam = rng.uniform(0.0, 8.0, (n_tri, per_tri, 1))
        o = X - lam * (-lv)[None, None, :]  # the ray o + t (-l.v) reaches X at t = lam
    else:
        lam = rng.uniform(0.0, 1.0, (n_tri, per_tri, 1))
        o = X + lam * (X - lv)               # the ray toward the light passes X
    o = o.reshape(-1, 3)
    lo, hi = v.reshape(-1, 3).min(0), v.reshape(-1, 3).max(0)
    c, R = 0.5 * (lo + hi), 0.5 * (hi - lo).max()
    inside = (np.abs(o - c) <= R).all(axis=1)
    return o[inside].astype(np.float32)
