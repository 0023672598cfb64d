#!/usr/bin/env python3
"""Per-launch HBM traffic of each render kernel from rocprofv3 --pmc passes.

    rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch -o fetch --output-format csv \\
        -- python3 bench.py --no-cpu ...
    rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write -o write --output-format csv \\
        -- python3 bench.py --no-cpu ...
    python tools/pmc_traffic.py gpurun_out/pmc_fetch gpurun_out/pmc_write -o profiles/x.json

FETCH_SIZE / WRITE_SIZE are in KiB (rocprofv3 derived counters), taken from
separate passes as MI355X_MICROARCH.md prescribes (FETCH_SIZE uses 3 of the
4 TCC slots, WRITE_SIZE 2).  On gfx950 FETCH_SIZE reports half the bytes of
wide coalesced (16 B/lane) streaming reads and is uncalibrated for other
shapes; the kernels mix coalesced staged fetches with scattered per-lane
float4 loads, so the raw count (x1) is the lower bound and x2 the upper one;
WRITE_SIZE is used as is.  Output: {kernel: {...}} per kernel family
(tools/pmc_reduce.py).
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_reduce import reduce_dir  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch_dir")
    ap.add_argument("write_dir", nargs="?")
    ap.add_argument("-o", "--out", required=True)
    a = ap.parse_args()
    f = reduce_dir(a.fetch_dir)
    w = reduce_dir(a.write_dir) if a.write_dir else {}
    out = {}
    for k, v in f.items():
        if "FETCH_SIZE" not in v:
            continue
        fk = v["FETCH_SIZE"]
        e = {"dispatches": v["dispatches"], "fetch_size_kib_raw": fk,
             "fetch_bytes_per_launch_lo": fk * 1024, "fetch_bytes_per_launch_hi": fk * 2048,
             "correction": "FETCH_SIZE KiB x1024 (lower bound) .. x2048 (upper bound: gfx950 "
                           "half-count of wide coalesced reads)"}
        wb = w.get(k, {}).get("WRITE_SIZE")
        if wb is not None:
            e["write_size_kib_raw"] = wb
            e["write_bytes_per_launch"] = wb * 1024
        e["hbm_bytes_per_launch"] = e["fetch_bytes_per_launch_lo"] + e.get("write_bytes_per_launch", 0.0)
        e["hbm_bytes_per_launch_hi"] = e["fetch_bytes_per_launch_hi"] + e.get("write_bytes_per_launch", 0.0)
        out[k] = e
    os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
    with open(a.out, "w") as fh:
        json.dump(out, fh, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
