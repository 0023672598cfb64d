#!/usr/bin/env python3
"""Per-call kernel timeline of rt_hip_cand_produce from a rocprofv3 kernel
trace of tools/prof_produce.py (not part of the product).

    python tools/produce_timeline.py prod_kernel_trace.csv --n 8 --steps 20
"""
import argparse
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--n", type=int, default=8)
    ap.add_argument("--steps", type=int, default=20)
    a = ap.parse_args()
    rows = sorted(csv.DictReader(open(a.csv)), key=lambda r: int(r["Start_Timestamp"]))
    names = [r["Kernel_Name"].split("(")[0].replace("void ", "")[:64] for r in rows]
    q = [i for i, n in enumerate(names) if "quick_kernel" in n]
    # calls: n warm-ups, then steps per rank
    for rank in (0, a.n - 1):
        ci = a.n + rank * a.steps + a.steps // 2
        if ci + 1 >= len(q):
            continue
        b0, b1 = q[ci], q[ci + 1]
        t0 = int(rows[b0]["Start_Timestamp"])
        busy = 0
        print(f"-- rank {rank} (call {ci})")
        for i in range(b0, b1):
            s, e = int(rows[i]["Start_Timestamp"]), int(rows[i]["End_Timestamp"])
            busy += e - s
            print(f"{(s - t0) / 1e3:8.1f} {(e - s) / 1e3:7.1f}  {names[i]}")
        end = int(rows[b1 - 1]["End_Timestamp"])
        print(f"span {(end - t0) / 1e3:.1f} us, kernels {busy / 1e3:.1f} us, next call at "
              f"{(int(rows[b1]['Start_Timestamp']) - t0) / 1e3:.1f} us")
    consume_view(rows, names)


def consume_view(rows, names):
    u = [i for i, n in enumerate(names) if "unpack_kernel" in n]
    if len(u) < 3:
        return
    b0, b1 = u[len(u) // 2], u[len(u) // 2 + 1]
    t0 = int(rows[b0]["Start_Timestamp"])
    print("-- consume (rank 0)")
    for i in range(b0, b1):
        s, e = int(rows[i]["Start_Timestamp"]), int(rows[i]["End_Timestamp"])
        print(f"{(s - t0) / 1e3:8.1f} {(e - s) / 1e3:7.1f}  {names[i]}")
    print(f"span {(int(rows[b1 - 1]['End_Timestamp']) - t0) / 1e3:.1f} us")


if __name__ == "__main__":
    main()
