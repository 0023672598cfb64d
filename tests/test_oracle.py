"""The oracle (oracle/rt_oracle.c) is pinned against the reference's own output.

Every golden framebuffer in tests/golden/ was produced by the reference cpu/rt
sources compiled unmodified (oracle/_ref/rt_probe); the restatement must
reproduce each one bit for bit, and the query counters exactly.
"""
import os

import numpy as np
import pytest

from conftest import (case_id, golden_image, load_manifest_static, load_own_manifest,
                      own_golden_image, own_scene_path)

CASES = load_manifest_static()
OWN_CASES = load_own_manifest()


@pytest.mark.parametrize("case", CASES, ids=[case_id(c) for c in CASES])
def test_oracle_matches_reference_golden(case, built, scene_dir):
    import oracle as orc
    sc = orc.OracleScene(os.path.join(scene_dir, case["scene"] + ".svati"))
    sc.set_size(case["width"], case["height"])
    img, cnt = orc.render(sc, case["width"], case["height"], threads=0)
    gold = golden_image(case)
    assert np.array_equal(img.view(np.uint32), gold.view(np.uint32)), \
        f"{int((img != gold).any(axis=2).sum())} pixels differ"
    assert cnt["closest"] == case["closest"]
    assert cnt["shadow"] == case["shadow"]


def test_oracle_pixel_subset_equals_full_frame(built, scene_dir, manifest):
    import oracle as orc
    case = next(c for c in manifest if c["scene"] == "cube" and c["width"] == 96)
    sc = orc.OracleScene(os.path.join(scene_dir, "cube.svati"))
    sc.set_size(96, 54)
    rng = np.random.default_rng(7)
    pix = np.stack([rng.integers(0, 54, 200), rng.integers(0, 96, 200)], axis=1)
    sub, _ = orc.render(sc, 96, 54, pixels=pix, threads=3)
    gold = golden_image(case)
    assert np.array_equal(sub, gold[pix[:, 0], pix[:, 1]])


def test_color_ops_known_answers(built):
    """cpu/colors.c:3-49 edge behaviour: clamps, NaN pass-through."""
    import oracle as orc
    L = orc.lib()
    c = L.oracle_init_color(2.0, -1.0, 0.5)
    assert (c.r, c.g, c.b) == (255.0, 0.0, np.float32(0.5) * np.float32(255))
    a = orc.ColorS(200.0, 10.0, 0.0)
    s = L.oracle_color_add(a, orc.ColorS(100.0, 1.0, 0.0))
    assert (s.r, s.g, s.b) == (255.0, 11.0, 0.0)
    m = L.oracle_color_mul(orc.ColorS(255.0, 128.0, 0.0), 0.25)
    exp_g = np.float32(np.float32(np.float32(128.0) / np.float32(255)) * np.float32(0.25)) * np.float32(255)
    assert m.g == exp_g


@pytest.mark.parametrize("case", OWN_CASES, ids=[case_id(c) for c in OWN_CASES])
def test_oracle_matches_reference_on_own_scenes(case, built, tmp_path):
    """Our own scenes (tests/golden/make_golden_own.py), rendered by the
    reference cpu/rt: two facing Nr 0.9 mirrors make every camera ray's path
    44 closest-hit queries deep (cpu/raytracer.c:19-34 recurses while coef >=
    0.01; 0.9^44 < 0.01)."""
    import oracle as orc
    sc = orc.OracleScene(own_scene_path(case, tmp_path))
    img, cnt = orc.render(sc, case["width"], case["height"], threads=0)
    assert np.array_equal(img.view(np.uint32), own_golden_image(case).view(np.uint32))
    assert cnt["closest"] == case["closest"] and cnt["shadow"] == case["shadow"]
    assert cnt["max_depth"] >= 43
