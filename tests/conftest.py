"""Shared fixtures.  GPU tests carry @pytest.mark.gpu; everything else runs on CPU.

Scenes: tests/golden/scenes/*.svati.gz are the reference's own test scenes
(data, gzipped).  Goldens: tests/golden/*.f32.gz + manifest.json, produced by
tests/golden/make_golden.py from the reference cpu/rt sources.
"""
import gzip
import json
import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(REPO, "tests", "golden")
sys.path.insert(0, os.path.join(REPO, "raytracing-gpu_amd"))
sys.path.insert(0, os.path.join(REPO, "oracle"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU")


@pytest.fixture(scope="session")
def built():
    """Bring the product library and the oracle up to date once per session
    (incremental make: a no-op when the in-tree build matches the sources)."""
    import oracle as orc
    import rtgpu
    rtgpu.build()
    orc.build()
    orc.lib()
    return True


@pytest.fixture(scope="session")
def scene_dir(tmp_path_factory):
    d = tmp_path_factory.mktemp("scenes")
    src = os.path.join(GOLDEN, "scenes")
    for f in os.listdir(src):
        if f.endswith(".svati.gz"):
            with gzip.open(os.path.join(src, f), "rb") as i, open(d / f[:-3], "wb") as o:
                o.write(i.read())
    return str(d)


@pytest.fixture(scope="session")
def manifest():
    with open(os.path.join(GOLDEN, "manifest.json")) as f:
        return json.load(f)["cases"]


def golden_image(case):
    with gzip.open(os.path.join(GOLDEN, case["file"]), "rb") as f:
        data = f.read()
    return np.frombuffer(data, dtype=np.float32).reshape(case["height"], case["width"], 3)


def case_id(case):
    return f'{case["scene"]}_{case["width"]}x{case["height"]}'


def load_manifest_static():
    with open(os.path.join(GOLDEN, "manifest.json")) as f:
        return json.load(f)["cases"]


OWN = os.path.join(GOLDEN, "own")


def load_own_manifest():
    """Goldens of our own scenes, rendered by the reference cpu/rt
    (tests/golden/make_golden_own.py)."""
    with open(os.path.join(OWN, "manifest.json")) as f:
        return json.load(f)["cases"]


def own_scene_path(case, tmpdir):
    """The case's .svati, unpacked into tmpdir."""
    dst = os.path.join(str(tmpdir), case["svati"][:-3])
    with gzip.open(os.path.join(OWN, case["svati"]), "rb") as i, open(dst, "wb") as o:
        o.write(i.read())
    return dst


def own_golden_image(case):
    with gzip.open(os.path.join(OWN, case["file"]), "rb") as f:
        data = f.read()
    return np.frombuffer(data, dtype=np.float32).reshape(case["height"], case["width"], 3)
