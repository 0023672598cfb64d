#!/usr/bin/env python3
"""Per-launch averages of rocprofv3 --pmc counters for each render kernel.

    python tools/pmc_reduce.py <rocprofv3 -d dir> -o out.json

Reads every *counter_collection.csv under the directory and averages each
counter over the dispatches of each kernel family: trace_kernel,
shade_kernel (the uninstrumented "false" instantiations: the instrumented
COUNT pass runs once per bench and is not part of the timed frames),
fold_kernel and the candidate-list kernels (by their own names).  Output:
{kernel: {counter: value per launch, "dispatches": n}}.
"""
import argparse
import collections
import csv
import glob
import json
import os
import re
import sys


def family(name):
    """Kernel family of a rocprofv3 Kernel_Name, None for instrumented passes."""
    m = re.search(r"(trace_kernel|shade_kernel|render_kernel)", name)
    if m:
        return m.group(1) if "false" in name else None
    m = re.search(r"rtc::(\w+_kernel)|rt::(\w+_kernel)", name)
    if m:
        return m.group(1) or m.group(2)
    return None


def reduce_dir(d):
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        sys.exit(f"no counter_collection.csv under {d}")
    for f in files:
        with open(f, newline="") as fh:
            for r in csv.DictReader(fh):
                k = family(r.get("Kernel_Name", ""))
                if not k:
                    continue
                acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
                disp[k].add(r.get("Dispatch_Id") or r.get("Correlation_Id"))
    out = {}
    for k, cs in acc.items():
        n = max(1, len(disp[k]))
        out[k] = {c: v / n for c, v in sorted(cs.items())}
        out[k]["dispatches"] = len(disp[k])
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("-o", "--out", required=True)
    a = ap.parse_args()
    res = reduce_dir(a.dir)
    with open(a.out, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
