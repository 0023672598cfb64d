#!/usr/bin/env python3
"""Per-launch HBM traffic of the render kernel from a rocprofv3 --pmc pass.

    rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch -o fetch --output-format csv \
        -- python3 bench.py --no-cpu ...
    rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write -o write --output-format csv \
        -- python3 bench.py --no-cpu ...
    python tools/pmc_traffic.py gpurun_out/pmc_fetch gpurun_out/pmc_write -o profiles/x.json

FETCH_SIZE / WRITE_SIZE are in KiB (rocprofv3 derived counters).  On gfx950
FETCH_SIZE reports half the bytes of wide coalesced (16 B/lane) streaming
reads (MI355X_MICROARCH.md "HBM") and is uncalibrated for other shapes.  The
render kernel mixes coalesced staged fetches with scattered per-lane float4
loads, so the raw count (x1) is reported as the lower bound and x2 as the
upper one; WRITE_SIZE is used as is.
Only dispatches of the uninstrumented render kernel (render_kernel<A, false>)
are averaged.
"""
import argparse
import csv
import glob
import json
import os
import sys


def rows(d):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        sys.exit(f"no counter_collection.csv under {d}")
    for f in files:
        with open(f, newline="") as fh:
            yield from csv.DictReader(fh)


def per_dispatch(d, counter, kernel_pat):
    acc = {}
    for r in rows(d):
        if r.get("Counter_Name") != counter:
            continue
        name = r.get("Kernel_Name", "")
        if kernel_pat not in name or "false" not in name:
            continue
        key = r.get("Dispatch_Id") or r.get("Correlation_Id")
        acc[key] = acc.get(key, 0.0) + float(r["Counter_Value"])
    return acc


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch_dir")
    ap.add_argument("write_dir", nargs="?")
    ap.add_argument("--kernel", default="render_kernel")
    ap.add_argument("-o", "--out", required=True)
    a = ap.parse_args()
    f = per_dispatch(a.fetch_dir, "FETCH_SIZE", a.kernel)
    if not f:
        sys.exit("no FETCH_SIZE rows for the render kernel")
    fetch_kib = sum(f.values()) / len(f)
    out = {"kernel": a.kernel, "dispatches": len(f),
           "fetch_size_kib_raw": fetch_kib,
           "fetch_bytes_per_launch_lo": fetch_kib * 1024,
           "fetch_bytes_per_launch_hi": fetch_kib * 1024 * 2,
           "correction": "FETCH_SIZE KiB x1024 (lower bound) .. x2048 (upper bound: gfx950 "
                         "half-count of wide coalesced reads)"}
    total = out["fetch_bytes_per_launch_lo"]
    if a.write_dir:
        w = per_dispatch(a.write_dir, "WRITE_SIZE", a.kernel)
        if w:
            wk = sum(w.values()) / len(w)
            out["write_size_kib_raw"] = wk
            out["write_bytes_per_launch"] = wk * 1024
            total += wk * 1024
    out["hbm_bytes_per_launch"] = total
    out["hbm_bytes_per_launch_hi"] = total + out["fetch_bytes_per_launch_lo"]
    os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
    with open(a.out, "w") as fh:
        json.dump(out, fh, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
