#!/usr/bin/env python3
"""Do two frames overlap on one GPU (not part of the product)?  Two
contexts of the C5 scene render on two HIP streams: N frames each one after
the other, then the same 2N frames issued alternately to the two streams.
If the second wall time is well below the first, a second frame's work
(e.g. the next frame's candidate lists) could hide in the first's tails.

    python3 tools/concurrency_probe.py --frames 10
"""
import argparse
import json
import os
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "raytracing-gpu_amd"))
import rtgpu  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=10)
    a = ap.parse_args()
    s = rtgpu.Scene.synthetic(32, 32, 9776, seed=0x5EED, width=3840, height=2160)
    f = s.frame()
    dev = torch.device("cuda", 0)
    per = rtgpu.tile_buffer_floats(f.width, f.height, 1)
    ctxs = [rtgpu.Context(s, "octree_gpu") for _ in range(2)]
    streams = [torch.cuda.Stream(device=dev) for _ in range(2)]
    bufs = [torch.empty(per, dtype=torch.float32, device=dev) for _ in range(2)]
    for c, st, b in zip(ctxs, streams, bufs):  # warm up: sizes, async shapes
        for _ in range(3):
            c.render(f, 0, 1, b.data_ptr(), st.cuda_stream)
        torch.cuda.synchronize()
        c.stats()
    res = {}
    torch.cuda.synchronize()
    t = time.perf_counter()
    for c, st, b in zip(ctxs, streams, bufs):
        for _ in range(a.frames):
            c.render(f, 0, 1, b.data_ptr(), st.cuda_stream)
        torch.cuda.synchronize()
    res["sequential_ms_per_frame"] = (time.perf_counter() - t) / (2 * a.frames) * 1e3
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(a.frames):
        for c, st, b in zip(ctxs, streams, bufs):
            c.render(f, 0, 1, b.data_ptr(), st.cuda_stream)
    torch.cuda.synchronize()
    res["two_streams_ms_per_frame"] = (time.perf_counter() - t) / (2 * a.frames) * 1e3
    for c in ctxs:
        c.stats()
    print(json.dumps(res))


if __name__ == "__main__":
    main()
