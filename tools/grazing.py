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


def grazing_rays(tri, n_tri, per_tri, seed=2, surface_frac=0.5):
    """Adversarial reflection-like rays: for n_tri random triangles, points X
    around each (barycentrics in [-0.5, 1.5]) and directions tilted out of
    the triangle's plane by a log-uniform 1e-7 .. 3e-2 rad -- rays that cross
    the plane right at the triangle at the most grazing angles, where the
    float Moller-Trumbore test's error region is largest.
    Origins: on the ray's line 0.01 .. 4 scene radii before X, or (a fraction
    surface_frac) ON another random triangle, as a reflection ray's origin is
    -- the direction then aims at X and only the crossing angle is grazing
    by construction when the two points are close to X's plane.  Kept inside
    the scene cube."""
    rng = np.random.default_rng(seed)
    v = tri[:, :3].astype(np.float64)
    v0, e1, e2 = v[:, 0], v[:, 1] - v[:, 0], v[:, 2] - v[:, 0]
    nrm = np.cross(e1, e2)
    nl = np.linalg.norm(nrm, axis=1)
    cand = np.flatnonzero(nl > 0)
    pick = rng.choice(cand, size=min(n_tri, len(cand)), replace=False)
    m = len(pick) * per_tri
    P = np.repeat(pick, per_tri)
    a = rng.uniform(-0.5, 1.5, (m, 1))
    b = rng.uniform(-0.5, 1.5, (m, 1))
    X = v0[P] + a * e1[P] + b * e2[P]
    n = nrm[P] / nl[P][:, None]
    # a random direction in the plane, tilted by theta
    t = rng.normal(size=(m, 3))
    t -= (t * n).sum(1)[:, None] * n
    t /= np.linalg.norm(t, axis=1)[:, None]
    th = 10.0 ** rng.uniform(-7, np.log10(3e-2), (m, 1)) * rng.choice([-1.0, 1.0], (m, 1))
    d = np.cos(th) * t + np.sin(th) * n
    lo, hi = v.reshape(-1, 3).min(0), v.reshape(-1, 3).max(0)
    c, R = 0.5 * (lo + hi), 0.5 * (hi - lo).max()
    lam = R * 10.0 ** rng.uniform(-2, np.log10(4.0), (m, 1))
    o = X - lam * d
    # reflection-like: origin on another triangle, aimed through X
    srf = rng.uniform(size=m) < surface_frac
    Q = rng.choice(cand, size=int(srf.sum()))
    qa = rng.uniform(0, 1, (len(Q), 1))
    qb = rng.uniform(0, 1, (len(Q), 1)) * (1 - qa)
    o2 = v0[Q] + qa * e1[Q] + qb * e2[Q]
    d2 = X[srf] - o2
    o[srf] = o2
    d[srf] = d2 / np.maximum(np.linalg.norm(d2, axis=1)[:, None], 1e-30)
    inside = (np.abs(o - c) <= R).all(axis=1)
    return o[inside].astype(np.float32), d[inside].astype(np.float32)


def float_mt(tri, o, d):
    """The reference's float Moller-Trumbore test (cpu/hit.c:15-37, float32
    operation by operation, no contraction) of one ray against every
    triangle: (accepting triangle indices, their new_dist)."""
    f = np.float32
    v0 = tri[:, 0, :].astype(f)
    e1 = (tri[:, 1, :] - tri[:, 0, :]).astype(f)
    e2 = (tri[:, 2, :] - tri[:, 0, :]).astype(f)
    O = np.asarray(o, f)
    D = np.broadcast_to(np.asarray(d, f), e2.shape)

    def cross(a, b):
        return np.stack([a[:, 1] * b[:, 2] - a[:, 2] * b[:, 1], a[:, 2] * b[:, 0] - a[:, 0] * b[:, 2],
                         a[:, 0] * b[:, 1] - a[:, 1] * b[:, 0]], 1)

    def dot(a, b):
        return (a[:, 0] * b[:, 0] + a[:, 1] * b[:, 1]) + a[:, 2] * b[:, 2]

    with np.errstate(all="ignore"):
        h = cross(D, e2)
        a = dot(e1, h)
        ok = ~((a > f(-1e-7)) & (a < f(1e-7)))
        fa = f(1) / a
        s = O[None, :] - v0
        u = fa * dot(s, h)
        ok &= ~((u < 0) | (u > 1))
        q = cross(s, e1)
        v = fa * dot(D, q)
        ok &= ~((v < 0) | (u + v > 1))
        t = fa * dot(e2, q)
        ok &= t > f(1e-7)
    idx = np.flatnonzero(ok)

    def length(x):  # cpu/vector3.c: float squares and sums, sqrt in double
        return np.sqrt(((x[:, 0] * x[:, 0] + x[:, 1] * x[:, 1]) + x[:, 2] * x[:, 2]).astype(np.float64)).astype(f)
    dl = length(D[:1])[0]
    nd = D[0] / dl
    P = O[None, :] + nd[None, :] * (t[idx] * dl)[:, None]
    dist = length(P - O[None, :])
    return idx, dist


def coplanar_grazing(tri_k, o, d, cos_max=1e-4, rel_off=1e-4):
    """Is the ray (o, d) the residual-risk class of a float garbage hit on
    triangle tri_k (DESIGN.md §2 "Reflection rays"): nearly IN the
    triangle's plane -- direction within cos_max of parallel and origin within
    rel_off (|o - v0| + 1) of the plane?  The float test can accept such a
    triangle from anywhere in its plane (a, s.h, d.q are all rounding noise)."""
    v = tri_k[:3].astype(np.float64)
    n = np.cross(v[1] - v[0], v[2] - v[0])
    n /= np.linalg.norm(n)
    dd = np.asarray(d, np.float64)
    c = abs(n @ dd) / np.linalg.norm(dd)
    off = abs(n @ (np.asarray(o, np.float64) - v[0]))
    return c < cos_max and off < rel_off * (np.linalg.norm(np.asarray(o, np.float64) - v[0]) + 1.0)
