#!/usr/bin/env python3
"""Per-rank trace cost of candidate tile -> rank maps, from one measured
per-tile cost map (tools/tile_cost.py --npy at N = 1, scanline tile order).
Not part of the product: it picks the map csrc/rt_tiles.h implements.

    python tools/tile_map_sim.py gpurun_out/r07a/tile_cost_n1.npz [--W 3840 --H 2160]

Maps (blocks of 4x4 tiles, block b in scanline order, blocks_x per row):
  mod      rank = b mod N                          (round 3-4)
  rot      rank = (b mod N + b div N) mod N        (each run of N blocks holds
                                                    one block per rank, rotated
                                                    by the run's index)
  diag     rank = (bx + by) mod N
  hash     rank = (b mod N + h(b div N)) mod N, h a multiplicative hash
"""
import argparse
import json

import numpy as np


def ranks_of(name, bx, by, blocks_x, n):
    b = by * blocks_x + bx
    if name == "mod":
        return b % n
    if name == "rot":
        return (b % n + b // n) % n
    if name == "diag":
        return (bx + by) % n
    if name == "hash":
        g = (b // n).astype(np.uint64)
        h = ((g * np.uint64(2654435761)) >> np.uint64(16)) % np.uint64(n)
        return (b % n + h.astype(np.int64)) % n
    raise ValueError(name)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("npz")
    ap.add_argument("--W", type=int, default=3840)
    ap.add_argument("--H", type=int, default=2160)
    a = ap.parse_args()
    d = np.load(a.npz)
    c, tx, ty = d["cycles"], d["tx"].astype(np.int64), d["ty"].astype(np.int64)
    ent = d["entries"] if d["entries"].size else None
    tb = 4
    tiles_x = (a.W + 7) // 8
    blocks_x = (tiles_x + tb - 1) // tb
    bx, by = tx // tb, ty // tb
    res = {}
    for n in (2, 4, 8):
        for name in ("mod", "rot", "diag", "hash"):
            rk = ranks_of(name, bx, by, blocks_x, n)
            per = np.bincount(rk, weights=c, minlength=n)
            e = {"max_over_mean": round(float(per.max() / per.mean()), 4),
                 "min_over_mean": round(float(per.min() / per.mean()), 4),
                 "tiles": np.bincount(rk, minlength=n).tolist()}
            if ent is not None:
                pe = np.bincount(rk, weights=ent, minlength=n)
                e["entries_max_over_mean"] = round(float(pe.max() / pe.mean()), 4)
            res[f"N{n}_{name}"] = e
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
