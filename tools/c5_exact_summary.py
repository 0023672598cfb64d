#!/usr/bin/env python3
"""Merge the parts of a whole-frame C5 parity run (tools/c5_exact.py over
disjoint rank ranges of one split) into one summary (not part of the product).

    python tools/c5_exact_summary.py gpurun_out/c5_exact_r05z_{a,b,c,d}.json -o summary.json
"""
import argparse
import json

ap = argparse.ArgumentParser()
ap.add_argument("parts", nargs="+")
ap.add_argument("-o", "--out", required=True)
ap.add_argument("--commit", default="")
a = ap.parse_args()
tot = {"pixels_compared": 0, "differing_pixels": 0, "differing_pixels_without_candidate_lists": 0, "ranks": []}
meta = None
for p in a.parts:
    d = json.load(open(p))
    meta = meta or {k: d[k] for k in ("grid", "tris", "W", "H", "accel", "nranks")}
    tot["pixels_compared"] += d["pixels_compared"]
    tot["differing_pixels"] += len(d["differ"])
    tot["differing_pixels_without_candidate_lists"] += d["differ_no_cand"]
    tot["ranks"] += d["ranks"]
ranks = sorted(set(tot["ranks"]))
out = {"what": "C5 %dx%d, %s (default: camera candidate lists + proven light buffers) vs brute force "
               "(RT_ACCEL_FLAT), every tile of %d of %d ranks of a %d-way split"
               % (meta["W"], meta["H"], meta["accel"], len(ranks), meta["nranks"], meta["nranks"]),
       "commit": a.commit, "frame_pixels": meta["W"] * meta["H"], "ranks_covered": len(ranks),
       "pixels_compared": tot["pixels_compared"], "differing_pixels": tot["differing_pixels"],
       "differing_pixels_without_candidate_lists": tot["differing_pixels_without_candidate_lists"],
       "parts": a.parts}
json.dump(out, open(a.out, "w"), indent=1)
print(json.dumps(out, indent=1))
