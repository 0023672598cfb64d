#!/usr/bin/env python3
"""Summary of a tools/rank_share.py run: per N the per-rank trace / shade
ranges, trace max / mean (the tile map's balance) and the slowest rank's
frame with per-rank and with triangle-parallel lists."""
import json
import sys

rows = json.load(open(sys.argv[1]))
for n in sorted({r["nranks"] for r in rows}):
    rs = [r for r in rows if r["nranks"] == n]
    tr = [r["trace_ms"] for r in rs]
    sh = [r["shade_ms"] for r in rs]
    line = {"N": n, "trace": [min(tr), max(tr)], "trace_max_over_mean": round(max(tr) / (sum(tr) / len(tr)), 4),
            "shade": [min(sh), max(sh)], "slowest_rank_lists": max(r["frame_ms"] for r in rs)}
    if all("partition" in r for r in rs):
        line["slowest_rank_partition"] = max(r["partition"]["frame_ms_without_exchange"] for r in rs)
        line["produce_max"] = max(r["partition"]["produce_ms_max"] for r in rs)
    print(json.dumps(line))
