#!/usr/bin/env python3
"""Host I/O of the drop-in path at C5 size:
the C5 scene written as .svati and .obj, loaded back with 1 and N host
threads (RT_HOST_THREADS), and a 3840x2160 P3 image written with 1 and N
threads.  Every multi-threaded result is checked byte-identical to the
single-threaded one.  Runs on the host only (no GPU needed).

    python tools/io_bench.py [--threads 16] [--dir /tmp] [--out gpurun_out/io_bench.json]
"""
import argparse
import hashlib
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "raytracing-gpu_amd"))
import rtgpu  # noqa: E402


def md5(path):
    h = hashlib.md5()
    with open(path, "rb") as f:
        for b in iter(lambda: f.read(1 << 24), b""):
            h.update(b)
    return h.hexdigest()


def timed(fn):
    t = time.perf_counter()
    r = fn()
    return r, time.perf_counter() - t


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--dir", default="/tmp")
    ap.add_argument("--grid", type=int, default=32)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    res = {"threads": a.threads, "host_cpus": os.cpu_count()}
    scene, t = timed(lambda: rtgpu.Scene.synthetic(a.grid, a.grid, 9776, seed=0x5EED,
                                                   width=3840, height=2160))
    res["triangles"] = scene.triangle_count
    res["generate_s"] = round(t, 3)
    paths = {"svati": os.path.join(a.dir, "c5_io.svati"), "obj": os.path.join(a.dir, "c5_io.obj")}
    try:
        for kind, p in paths.items():
            row = {}
            wh = {}
            for nt in (1, a.threads):
                os.environ["RT_HOST_THREADS"] = str(nt)
                _, t = timed(lambda: getattr(scene, "write_" + kind)(p))
                size = os.path.getsize(p)
                wh[nt] = md5(p)
                row["bytes"] = size
                row[f"write_s_{nt}t"] = round(t, 3)
                row[f"write_GBps_{nt}t"] = round(size / t / 1e9, 3)
            row["write_identical"] = wh[1] == wh[a.threads]
            row["write_speedup"] = round(row["write_s_1t"] / row[f"write_s_{a.threads}t"], 2)
            ref = None
            for nt in (1, a.threads):
                os.environ["RT_HOST_THREADS"] = str(nt)
                s2, t = timed(lambda: getattr(rtgpu.Scene, "load_" + kind)(p))
                row[f"load_s_{nt}t"] = round(t, 3)
                row[f"load_GBps_{nt}t"] = round(size / t / 1e9, 3)
                # the loaded scene written back: identical bytes for every thread count
                back = p + f".back{nt}"
                getattr(s2, "write_" + kind)(back)
                h = md5(back)
                os.remove(back)
                ref = ref or h
                row[f"roundtrip_identical_{nt}t"] = h == ref
                assert s2.triangle_count == scene.triangle_count
                del s2
            row["load_speedup"] = round(row["load_s_1t"] / row[f"load_s_{a.threads}t"], 2)
            res[kind] = row
            print(kind, json.dumps(row), flush=True)
    finally:
        for p in paths.values():
            if os.path.exists(p):
                os.remove(p)
    # 4K P3 output (cpu/printer.c:12-18): a deterministic non-trivial image
    rng = np.random.default_rng(7)
    img = (rng.random((2160, 3840, 3), dtype=np.float32) * 255.0).astype(np.float32)
    ppm = os.path.join(a.dir, "c5_io.ppm")
    row = {}
    hashes = {}
    for nt in (1, a.threads):
        os.environ["RT_HOST_THREADS"] = str(nt)
        _, t = timed(lambda: rtgpu.write_ppm(ppm, img))
        size = os.path.getsize(ppm)
        hashes[nt] = md5(ppm)
        row[f"write_s_{nt}t"] = round(t, 3)
        row[f"write_GBps_{nt}t"] = round(size / t / 1e9, 3)
        row["bytes"] = size
    os.remove(ppm)
    row["identical"] = hashes[1] == hashes[a.threads]
    row["speedup"] = round(row["write_s_1t"] / row[f"write_s_{a.threads}t"], 2)
    res["ppm_4k"] = row
    print("ppm", json.dumps(row), flush=True)
    if a.out:
        os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
