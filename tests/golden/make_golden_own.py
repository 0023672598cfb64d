#!/usr/bin/env python3
"""Golden fixtures for scenes of our own, rendered by the *reference* cpu/rt
(build container only; TEST INFRASTRUCTURE, like make_golden.py).

The reference ships no scene that exercises cpu/rt's unbounded reflection
recursion (cpu/raytracer.c:19-34): its deepest measured path is 7 bounces.
`mirrors` is two facing Nr 0.9 mirror quads, 0.9^k < 0.01 first at k = 44,
so paths reach 44 closest-hit queries -- beyond the 32-term buffer that
round 2's render kernel refused with RT_EDEPTH.  The scene text is
generated here (our data), rendered by oracle/_ref/rt_probe (the reference's
cpu/ sources compiled unmodified by oracle/Makefile), and stored as
tests/golden/own/<scene>.svati.gz + <scene>_<W>x<H>.f32.gz + manifest.json.

    python tests/golden/make_golden_own.py
"""
import gzip
import hashlib
import json
import os
import re
import subprocess
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
PROBE = os.path.join(REPO, "oracle", "_ref", "rt_probe")
OUT = os.path.join(HERE, "own")


def quad(z, half, normal_z):
    """Two triangles of the square |x|, |y| <= half at depth z (6 v + 6 vn lines)."""
    v = [(-half, -half, z), (half, -half, z), (half, half, z),
         (-half, -half, z), (half, half, z), (-half, half, z)]
    lines = [f"v {x} {y} {zz}" for x, y, zz in v]
    lines += [f"vn 0 0 {normal_z}"] * 6
    return lines


def mirrors(w, h):
    # camera at the origin, u = +x, v = -y, fov 40: w = u x v = -z, so the
    # film plane sits at z = -L, L = w / (2 tan 20 deg), and camera rays run
    # from it through the eye towards +z (cpu/raytracer.c:82-86, SURVEY.md
    # Appendix A item 10).  Mirror A at z = +5 faces the eye, mirror B sits
    # behind the film at z = -(L + 5): every camera ray bounces between them.
    L = w / (2 * 0.36397023426620234)
    zb = round(L + 5.0, 3)
    obj = []
    for z, nz in ((5.0, -1), (-zb, 1)):
        obj += ["object 6", "Ka 0.05 0.04 0.03", "Kd 0.4 0.5 0.6", "Ks 0.3 0.3 0.3", "Ns 12",
                "Nr 0.9"] + quad(z, 4000.0, nz) + [""]
    return "\n".join([f"camera {w} {h} 0 0 0 1 0 0 0 -1 0 40", "a_light 0.3 0.3 0.3",
                      "d_light 1 0.9 0.8 0.2 -0.3 -1", "p_light 0.5 0.5 0.5 3 2 1", ""] + obj)


SCENES = {"mirrors": (mirrors, [(32, 18), (96, 54)])}


def main():
    os.makedirs(OUT, exist_ok=True)
    cases = []
    for name, (gen, sizes) in SCENES.items():
        for w, h in sizes:
            text = gen(w, h)
            with tempfile.TemporaryDirectory() as td:
                sv = os.path.join(td, f"{name}.svati")
                with open(sv, "w") as f:
                    f.write(text)
                dump, ppm = os.path.join(td, "o.f32"), os.path.join(td, "o.ppm")
                p = subprocess.run(["bash", "-c", f"ulimit -s unlimited && exec {PROBE} {sv} {dump}"],
                                   env=dict(os.environ, RT_PROBE_PPM=ppm), capture_output=True,
                                   text=True, check=True)
                m = re.search(r"closest_hit_queries=(\d+) shadow_queries=(\d+)", p.stderr)
                with open(dump, "rb") as f:
                    assert f.readline() == f"RTF32 {w} {h}\n".encode()
                    data = f.read()
                with open(ppm, "rb") as f:
                    ppm_md5 = hashlib.md5(f.read()).hexdigest()
            sname = f"{name}_{w}x{h}.svati.gz"
            with open(os.path.join(OUT, sname), "wb") as raw:
                with gzip.GzipFile(fileobj=raw, mode="wb", compresslevel=9, mtime=0) as f:
                    f.write(text.encode())
            fname = f"{name}_{w}x{h}.f32.gz"
            with open(os.path.join(OUT, fname), "wb") as raw:
                with gzip.GzipFile(fileobj=raw, mode="wb", compresslevel=9, mtime=0) as f:
                    f.write(data)
            cases.append({"scene": name, "width": w, "height": h, "svati": sname, "file": fname,
                          "closest": int(m.group(1)), "shadow": int(m.group(2)),
                          "f32_sha256": hashlib.sha256(data).hexdigest(), "ppm_md5": ppm_md5})
            print(cases[-1])
    with open(os.path.join(OUT, "manifest.json"), "w") as f:
        json.dump({"generator": "tests/golden/make_golden_own.py (reference cpu/rt via oracle/_ref/rt_probe)",
                   "cases": cases}, f, indent=1)


if __name__ == "__main__":
    main()
