#!/usr/bin/env python3
"""Forward error bound of the reference's float Moller-Trumbore test
(/root/reference/cpu/hit.c:15-33), and a stress check of it.

The reference computes, in float and in this order (no FMA):
    h = d x e2; a = e1.h; reject |a| < 1e-7f; f = 1/a; s = o - v0;
    u = f (s.h); q = s x e1; v = f (d.q); t = f (e2.q)
With eps = 2^-24 (unit roundoff), |S| = |o - v0| (exact), |d|, |e1|, |e2|,
the float s.h, d.q, e2.q and a differ from their exact values by at most
    E_sh = C_DOT eps |S| |d| |e2|     E_dq = C_DOT eps |S| |d| |e1|
    E_eq = C_DOT eps |S| |e1| |e2|    E_a  = C_A eps |e1| |d| |e2|
(componentwise rounding of s, h, q, of each product and of the two sums,
bounded with Cauchy-Schwarz; C_DOT = 6 sqrt 2 = 8.49 -> 8.6, C_A = 5 sqrt 2
= 7.07 -> 7.2).  So a float accept (u, v in [0,1], u + v <= 1) implies the
exact barycentrics U = S.H/A, V = d.Q/A of the exact line's plane crossing
satisfy U >= -du, V >= -dv, U + V <= 1 + dw with
    rho = E_a / a_lb,  du = E_sh / (a_lb (1 - rho)),  dv = E_dq / (a_lb (1 - rho)),
    dw = (4 eps + (E_sh + E_dq) / a_lb + rho) / (1 - rho)
for any lower bound a_lb <= |a| (at least 1e-7f, since smaller |a| is
rejected).  csrc/rt_cand.hip evaluates exactly these formulas per triangle
for the camera rays; this script checks them against the
float test itself on grazing rays.

    python tools/mt_bound.py [--n 2000000]
"""
import argparse

import numpy as np

EPS = 2.0 ** -24
C_DOT = 8.6
C_A = 7.2
A_MIN = float(np.float32(1e-7))  # the reference's reject threshold (float)


def mt_f32(o, d, v0, e1, e2):
    """The reference's float test, vectorised (numpy float32 = IEEE, no FMA)."""
    f32 = np.float32
    o, d, v0, e1, e2 = (np.asarray(x, f32) for x in (o, d, v0, e1, e2))

    def cross(a, b):
        return np.stack([a[:, 1] * b[:, 2] - a[:, 2] * b[:, 1],
                         a[:, 2] * b[:, 0] - a[:, 0] * b[:, 2],
                         a[:, 0] * b[:, 1] - a[:, 1] * b[:, 0]], axis=1)

    def dot(a, b):
        return (a[:, 0] * b[:, 0] + a[:, 1] * b[:, 1]) + a[:, 2] * b[:, 2]

    eps = f32(1e-7)
    with np.errstate(all="ignore"):
        h = cross(d, e2)
        a = dot(e1, h)
        ok = ~((a > -eps) & (a < eps))
        f = f32(1) / a
        s = o - v0
        u = f * dot(s, h)
        ok &= ~((u < 0) | (u > 1))
        q = cross(s, e1)
        v = f * dot(d, q)
        ok &= ~((v < 0) | (u + v > 1))
        t = f * dot(e2, q)
        ok &= t > eps
    return ok, u, v, t


def bound(S, dlen, l1, l2, a_lb):
    """(du, dv, dw) of the module docstring; inf when rho >= 1/2."""
    e_sh = C_DOT * EPS * S * dlen * l2
    e_dq = C_DOT * EPS * S * dlen * l1
    e_a = C_A * EPS * l1 * dlen * l2
    rho = e_a / a_lb
    bad = rho >= 0.5
    with np.errstate(all="ignore"):
        du = np.where(bad, np.inf, e_sh / (a_lb * (1 - rho)))
        dv = np.where(bad, np.inf, e_dq / (a_lb * (1 - rho)))
        dw = np.where(bad, np.inf, (4 * EPS + (e_sh + e_dq) / a_lb + rho) / (1 - rho))
    return du, dv, dw, e_a


def exact_bary(o, d, v0, e1, e2):
    o, d, v0, e1, e2 = (np.asarray(x, np.float64) for x in (o, d, v0, e1, e2))
    H = np.cross(d, e2)
    A = np.einsum("ij,ij->i", e1, H)
    S = o - v0
    U = np.einsum("ij,ij->i", S, H) / A
    Q = np.cross(S, e1)
    V = np.einsum("ij,ij->i", d, Q) / A
    return U, V, A


def bound_cw(o, d, v0, e1, e2, a_lb):
    """Componentwise version (csrc/rt_cand.hip second round):
    E_sh <= 6.01 eps sum |S_i| M_i, M_i = |d_j| |e2_k| + |d_k| |e2_j|;
    E_dq <= 6.01 eps sum |d_i| N_i, N_i = |S_j| |e1_k| + |S_k| |e1_j|;
    E_a <= 5.01 eps sum |e1_i| M_i.  Returns (du, dv, dw)."""
    D = np.abs(np.asarray(d, np.float64))
    S = np.abs(np.asarray(o, np.float64) - np.asarray(v0, np.float64))
    E1 = np.abs(np.asarray(e1, np.float64))
    E2 = np.abs(np.asarray(e2, np.float64))
    M = np.stack([D[:, 1] * E2[:, 2] + D[:, 2] * E2[:, 1], D[:, 2] * E2[:, 0] + D[:, 0] * E2[:, 2],
                  D[:, 0] * E2[:, 1] + D[:, 1] * E2[:, 0]], 1)
    N = np.stack([S[:, 1] * E1[:, 2] + S[:, 2] * E1[:, 1], S[:, 2] * E1[:, 0] + S[:, 0] * E1[:, 2],
                  S[:, 0] * E1[:, 1] + S[:, 1] * E1[:, 0]], 1)
    e_sh = 6.01 * EPS * (S * M).sum(1)
    e_dq = 6.01 * EPS * (D * N).sum(1)
    e_a = 5.01 * EPS * (E1 * M).sum(1)
    rho = e_a / a_lb
    with np.errstate(all="ignore"):
        du = e_sh / (a_lb * (1 - rho))
        dv = e_dq / (a_lb * (1 - rho))
        dw = (4 * EPS + (e_sh + e_dq) / a_lb + rho) / (1 - rho)
    bad = rho >= 0.5
    return np.where(bad, np.inf, du), np.where(bad, np.inf, dv), np.where(bad, np.inf, dw)


def stress(n, seed=1, far=2900.0, componentwise=False):
    """Grazing rays from far origins (like camera rays) at random
    well-shaped and sliver triangles; returns (accepts, violations, worst
    ratio of the observed error to the bound)."""
    rng = np.random.default_rng(seed)
    # triangles of edge ~0.06 (C5) and slivers
    v0 = rng.uniform(-40, 40, (n, 3)).astype(np.float32)
    ax = rng.normal(size=(n, 3))
    ax /= np.linalg.norm(ax, axis=1, keepdims=True)
    by = np.cross(ax, rng.normal(size=(n, 3)))
    by /= np.linalg.norm(by, axis=1, keepdims=True)
    ln = rng.uniform(0.02, 0.4, n)[:, None]
    wd = ln * rng.choice([1.0, 0.3, 0.05], n)[:, None]
    e1 = (ax * ln).astype(np.float32)
    e2 = (ax * ln * rng.uniform(0.2, 1.0, n)[:, None] + by * wd).astype(np.float32)
    nrm = np.cross(e1.astype(np.float64), e2.astype(np.float64))
    nrm /= np.linalg.norm(nrm, axis=1, keepdims=True)
    # a point of the extended plane near the triangle, a direction almost in
    # the plane (|cos| log-uniform in [1e-6, 0.3])
    tgt = v0 + rng.uniform(-3, 4, (n, 1)) * e1 + rng.uniform(-3, 4, (n, 1)) * e2
    inplane = np.cross(nrm, rng.normal(size=(n, 3)))
    inplane /= np.linalg.norm(inplane, axis=1, keepdims=True)
    c = 10 ** rng.uniform(-6, np.log10(0.3), n)
    dirn = inplane * np.sqrt(1 - c * c)[:, None] + nrm * (c * rng.choice([-1, 1], n))[:, None]
    o = (tgt - dirn * rng.uniform(0.3, 1.0, n)[:, None] * far).astype(np.float32)
    # the float direction as the reference builds camera rays: normalize(target - o)
    dv = (tgt.astype(np.float32) - o).astype(np.float32)
    ln2 = np.sqrt((dv.astype(np.float32) * dv).sum(axis=1, dtype=np.float32).astype(np.float64)).astype(np.float32)
    d = (dv / ln2[:, None]).astype(np.float32)
    ok, u, v, t = mt_f32(o, d, v0, e1, e2)
    U, V, A = exact_bary(o, d, v0, e1, e2)
    S = np.linalg.norm(o.astype(np.float64) - v0, axis=1)
    dlen = np.linalg.norm(d.astype(np.float64), axis=1)
    l1 = np.linalg.norm(e1.astype(np.float64), axis=1)
    l2 = np.linalg.norm(e2.astype(np.float64), axis=1)
    e_a = C_A * EPS * l1 * dlen * l2
    a_lb = np.maximum(A_MIN, np.abs(A) - e_a)
    if componentwise:
        du, dv_, dw = bound_cw(o, d, v0, e1, e2, a_lb)
    else:
        du, dv_, dw, _ = bound(S, dlen, l1, l2, a_lb)
    viol = ok & ((U < -du) | (V < -dv_) | (U + V > 1 + dw))
    with np.errstate(all="ignore"):
        ratio = np.max(np.where(ok, np.maximum.reduce([-U / du, -V / dv_, (U + V - 1) / dw]), 0))
    return int(ok.sum()), int(viol.sum()), float(ratio)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=2_000_000)
    ap.add_argument("--seeds", type=int, default=3)
    a = ap.parse_args()
    for cw in (False, True):
        for s in range(a.seeds):
            acc, viol, ratio = stress(a.n, seed=s, componentwise=cw)
            print(f"{'componentwise' if cw else 'Cauchy-Schwarz'} seed {s}: {acc} float accepts, "
                  f"{viol} outside the bound, worst error/bound {ratio:.3f}")


if __name__ == "__main__":
    main()
