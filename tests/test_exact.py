"""Exact camera rays (csrc/rt_cand.hip): the forward error
bound of the reference's float Moller-Trumbore test and the host mirror of
the per-frame candidate lists.  CPU only."""
import os
import sys

import numpy as np
import pytest

from conftest import REPO

sys.path.insert(0, os.path.join(REPO, "tools"))


@pytest.mark.parametrize("componentwise", [False, True])
def test_mt_error_bound_holds_on_grazing_rays(componentwise):
    """cpu/hit.c:15-33 in float on grazing rays from far origins: every float
    accept's exact plane crossing lies inside the expanded triangle of the
    bound (Cauchy-Schwarz and componentwise forms)."""
    import mt_bound
    acc, viol, ratio = mt_bound.stress(200_000, seed=11, componentwise=componentwise)
    assert acc > 2000
    assert viol == 0
    assert 0.0 < ratio < 1.0


def test_mt_f32_is_the_moller_trumbore_test():
    """The numpy float restatement computes the Moller-Trumbore barycentrics:
    on well-conditioned random rays its accept decisions are the exact ones."""
    import mt_bound
    rng = np.random.default_rng(5)
    n = 20000
    v0 = rng.uniform(-1, 1, (n, 3)).astype(np.float32)
    e1 = rng.uniform(-1, 1, (n, 3)).astype(np.float32)
    e2 = rng.uniform(-1, 1, (n, 3)).astype(np.float32)
    o = rng.uniform(-5, 5, (n, 3)).astype(np.float32)
    d = (v0 + 0.3 * e1 + 0.3 * e2 - o).astype(np.float32)
    ok, u, v, t = mt_bound.mt_f32(o, d, v0, e1, e2)
    assert ok.mean() > 0.5  # aimed at the triangles
    U, V, A = mt_bound.exact_bary(o, d, v0, e1, e2)
    inside = (U >= 0) & (V >= 0) & (U + V <= 1)
    margin = np.minimum(np.minimum(np.abs(U), np.abs(V)), np.abs(1 - U - V))
    well = (np.abs(A) > 1e-2) & (margin > 1e-3)
    assert well.sum() > n // 4
    assert np.array_equal(ok[well], inside[well])


def test_c5_tessellation_is_near_square():
    """C5 spheres: 53 stacks x 94 slices = 9776 triangles (round 1's 258 x 19
    slivers are still available through synthetic_uv)."""
    import rtgpu
    s = rtgpu.Scene.synthetic(1, 1, 9766, seed=0x5EED, width=64, height=36)
    assert s.triangle_count == 9776 + 2
    t = s.triangles_array()[2:, :3].astype(np.float64)
    e = np.linalg.norm(t[:, [1, 2, 0]] - t, axis=2)
    mid = t[len(t) // 2 - 200: len(t) // 2 + 200]
    em = np.linalg.norm(mid[:, [1, 2, 0]] - mid, axis=2)
    assert em.max(axis=1).max() / em.min(axis=1).min() < 4.0  # equator: no slivers
    old = rtgpu.Scene.synthetic_uv(1, 1, 258, 19, seed=0x5EED, width=64, height=36)
    assert old.triangle_count == 9766 + 2
    assert e.shape[0] == 9776


def test_candidate_survey_partitions_the_triangles():
    """Host mirror of the device classifier: every triangle is safe, listed
    or global; tighter bounds list fewer; the proven bound (scale 1) lists
    the most."""
    import rtgpu
    s = rtgpu.Scene.synthetic(4, 4, 1200, seed=0x5EED, width=480, height=270)
    n = s.triangle_count
    r1 = rtgpu.cand_survey(s, 64.0, 1.0)
    r2 = rtgpu.cand_survey(s, 64.0, 0.25)
    for r in (r1, r2):
        assert r["safe"] + r["footprint"] + r["global"] == n
        assert sum(h[2] for h in r["hist"]) == r["entries"]
    assert r2["safe"] >= r1["safe"] and r2["entries"] <= r1["entries"]
    assert r1["entries"] > 0
    r3 = rtgpu.cand_survey(s, 256.0, 1.0)  # more culling slack: fewer risky triangles
    assert r3["safe"] >= r1["safe"]
    assert rtgpu.cand_survey(s, 64.0, 1.0) == r1  # deterministic


def test_candidate_survey_reference_scene(scene_dir):
    """A reference scene with large triangles: almost everything is safe."""
    import rtgpu
    s = rtgpu.Scene.load_svati(os.path.join(scene_dir, "car-on-road.svati"))
    s.set_size(1920, 1080)
    r = rtgpu.cand_survey(s, 64.0, 1.0)
    assert r["safe"] + r["footprint"] + r["global"] == s.triangle_count


@pytest.mark.parametrize("case", ["small", "c5"])
def test_tile_refinement_drops_only_tiles_the_reference_never_accepts(case):
    """The per-tile refinement of the camera candidate lists (csrc/rt_cand.hip
    tile_keep) drops a (triangle, tile) entry only where its proof says no
    camera sample of the tile can pass the float test.  Checked against the
    oracle's restatement of cpu/hit.c:15-44 on every camera sample
    (cpu/raytracer.c:50-61) of the dropped tiles: none may pass even the a, u,
    v stages.  The kept entries include the tiles the triangle is really hit
    in (the geometry of the tile mapping and projection is right).  c5: the
    headline scene, every 200th refined entry."""
    import rtgpu
    import oracle as orc
    if case == "small":
        s = rtgpu.Scene.synthetic(4, 4, 1200, seed=0x5EED, width=480, height=270)
        stride = 1
    else:
        s = rtgpu.Scene.synthetic(32, 32, 9776, seed=0x5EED, width=3840, height=2160)
        stride = 200
    rows, total = rtgpu.cand_refine_sample(s, stride=stride, cap=1 << 20)
    assert len(rows) == total > 0
    drop = rows[:, 3] == 0
    assert drop.sum() > 0 and (~drop).sum() > 0
    tris = s.triangles_array()
    rects = np.stack([rows[:, 2] * 8, rows[:, 1] * 8, np.full(len(rows), 8), np.full(len(rows), 8)], 1)
    acc = orc.camera_tri_accepts(s.ptr, tris[rows[:, 0]], rects)
    assert int(acc[drop, 1].max()) == 0, rows[drop][acc[drop, 1] > 0][:8]
    assert int((acc[~drop, 0] > 0).sum()) > 0  # real hits live in kept tiles


def test_tile_refinement_compat_drops_only_never_accepted_tiles():
    """test_tile_refinement_drops_only_tiles_the_reference_never_accepts for
    the gpu/rt compatibility mode's lists (one ray per pixel of the 3x frame,
    gpu/raytracer.cu:97-103; tile_keep's compat sample rectangle), checked
    with the oracle's restatement of those rays."""
    import rtgpu
    import oracle as orc
    s = rtgpu.Scene.synthetic(4, 4, 1200, seed=0x5EED, width=160, height=90)
    rows, total = rtgpu.cand_refine_sample(s, stride=1, cap=1 << 20, compat=True)
    assert len(rows) == total > 0
    drop = rows[:, 3] == 0
    assert drop.sum() > 0 and (~drop).sum() > 0
    tris = s.triangles_array()
    rects = np.stack([rows[:, 2] * 8, rows[:, 1] * 8, np.full(len(rows), 8), np.full(len(rows), 8)], 1)
    acc = orc.camera_tri_accepts(s.ptr, tris[rows[:, 0]], rects, gpu=True)
    assert int(acc[drop, 1].max()) == 0, rows[drop][acc[drop, 1] > 0][:8]
    assert int((acc[~drop, 0] > 0).sum()) > 0
