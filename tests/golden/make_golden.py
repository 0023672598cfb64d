#!/usr/bin/env python3
"""Regenerate the golden fixtures from the *reference* cpu/rt (build container only).

TEST INFRASTRUCTURE.  Runs oracle/_ref/rt_probe -- the reference's own cpu/ sources
compiled unmodified by oracle/Makefile, with oracle/probe.c replacing printer.c --
on every scene in /root/reference/tests with the camera line's width/height
rewritten (the field of view is preserved), and stores:

  <scene>_<W>x<H>.f32.gz   W*H*3 float32 framebuffer in PPM order (bit-exact)
  manifest.json            per case: triangles, query counts, md5 of the P3 PPM

Only data (inputs' names and outputs) is committed; the reference's sources and
scene files are not.  Usage: python tests/golden/make_golden.py [--jobs N]
"""
import argparse
import concurrent.futures as cf
import gzip
import hashlib
import json
import os
import re
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF_TESTS = "/root/reference/tests"
PROBE = os.path.join(REPO, "oracle", "_ref", "rt_probe")

SMALL = (96, 54)
# (scene, W, H): the small sweep over every reference scene, plus config C1.
EXTRA = [("cube", 256, 256), ("triangle", 64, 64), ("island_smooth", 192, 108)]


def rewrite_camera(src, dst, w, h):
    out = []
    with open(src) as f:
        for line in f:
            fields = line.split()
            if fields and fields[0] == "camera":
                fields[1], fields[2] = str(w), str(h)
                line = " ".join(fields) + "\n"
            out.append(line)
    with open(dst, "w") as f:
        f.writelines(out)


def run_case(scene, w, h):
    with tempfile.TemporaryDirectory() as td:
        svati = os.path.join(td, f"{scene}.svati")
        rewrite_camera(os.path.join(REF_TESTS, f"{scene}.svati"), svati, w, h)
        dump = os.path.join(td, "out.f32")
        ppm = os.path.join(td, "out.ppm")
        env = dict(os.environ, RT_PROBE_PPM=ppm)
        p = subprocess.run(["bash", "-c", f"ulimit -s unlimited && exec {PROBE} {svati} {dump}"],
                           env=env, capture_output=True, text=True, check=True)
        m = re.search(r"closest_hit_queries=(\d+) shadow_queries=(\d+)", p.stderr)
        with open(dump, "rb") as f:
            header = f.readline()
            data = f.read()
        assert header == f"RTF32 {w} {h}\n".encode(), header
        assert len(data) == w * h * 12
        with open(ppm, "rb") as f:
            ppm_bytes = f.read()
    name = f"{scene}_{w}x{h}.f32.gz"
    with open(os.path.join(HERE, name), "wb") as raw:
        with gzip.GzipFile(fileobj=raw, mode="wb", compresslevel=9, mtime=0) as f:
            f.write(data)
    return {
        "scene": scene, "width": w, "height": h, "file": name,
        "closest": int(m.group(1)), "shadow": int(m.group(2)),
        "f32_sha256": hashlib.sha256(data).hexdigest(),
        "ppm_md5": hashlib.md5(ppm_bytes).hexdigest(),
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--jobs", type=int, default=2)
    args = ap.parse_args()
    if not os.path.exists(PROBE):
        sys.exit("build the reference probe first: make -C oracle ref")
    scenes = sorted(f[:-6] for f in os.listdir(REF_TESTS) if f.endswith(".svati"))
    cases = [(s, *SMALL) for s in scenes] + EXTRA
    with cf.ThreadPoolExecutor(args.jobs) as ex:
        results = list(ex.map(lambda c: run_case(*c), cases))
    with open(os.path.join(HERE, "manifest.json"), "w") as f:
        json.dump({"generator": "oracle/_ref/rt_probe (reference cpu/ sources, -O2, probe.c)",
                   "cases": results}, f, indent=1)
    for r in results:
        print(r["scene"], r["width"], r["height"], r["closest"], r["shadow"], r["ppm_md5"])


if __name__ == "__main__":
    main()
