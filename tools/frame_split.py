#!/usr/bin/env python3
"""Per-frame kernel times from a rocprofv3 kernel trace of bench.py (not part
of the product): frames are split at each trace_kernel dispatch (a frame's
list kernels come before its trace), and the kernels of the last N frames
(bench's fresh-camera loop) are compared with the N before them (the timed
replay loop).

    python3 tools/frame_split.py gpurun_out/x/run_kernel_trace.csv --frames 20
"""
import argparse
import csv
import collections


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--frames", type=int, default=20)
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    frames, cur = [], []
    for r in rows:
        name = r["Kernel_Name"].split("(")[0].replace("void ", "")
        dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        cur.append((name, dur, int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
        if "trace_kernel" in name:
            frames.append(cur)
            cur = []
    if cur and frames:
        frames[-1].extend(cur)  # shade / fold / fixups of the last frame
    # a frame's shade and fold come after its trace: move everything after
    # each trace up to the next list build into that frame -- approximated by
    # attaching shade/fold/oob kernels that precede the next frame's lists
    fixed = []
    carry = []
    for f in frames:
        head = [k for k in f if k[0].startswith(("rt::shade", "rt::fold", "rt::oob"))]
        rest = [k for k in f if not k[0].startswith(("rt::shade", "rt::fold", "rt::oob"))]
        if fixed:
            fixed[-1].extend(head)
        fixed.append(rest)
    n = a.frames
    fresh, replay = fixed[-n:], fixed[-2 * n:-n]

    def summary(fs):
        s = collections.defaultdict(float)
        for f in fs:
            for name, dur, _, _ in f:
                s[name] += dur / len(fs)
        return s

    def span(fs):
        return sum((f[-1][3] - f[0][2]) / 1e3 for f in fs if f) / len(fs)

    sr, sf = summary(replay), summary(fresh)
    print(f"frames: replay {len(replay)}, fresh {len(fresh)}; span per frame (us): replay {span(replay):.1f} "
          f"fresh {span(fresh):.1f}")
    keys = sorted(set(sr) | set(sf), key=lambda k: -(sf.get(k, 0) + sr.get(k, 0)))
    for k in keys:
        d = sf.get(k, 0) - sr.get(k, 0)
        print(f"{k[:70]:70s} {sr.get(k, 0):9.1f} {sf.get(k, 0):9.1f} {d:+8.1f}")
    print(f"{'total kernel time':70s} {sum(sr.values()):9.1f} {sum(sf.values()):9.1f}")


if __name__ == "__main__":
    main()
