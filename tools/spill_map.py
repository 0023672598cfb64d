#!/usr/bin/env python3
"""Where a kernel's scratch spills sit (innermost loop of each spill/reload
instruction in the gfx950 ISA).  Build-time analysis only.

    python tools/spill_map.py <mangled-kernel-substring> [-D...]
"""
import os
import re
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "raytracing-gpu_amd")


def main():
    key = sys.argv[1]
    src = os.path.join(PKG, "csrc", "rt_render.hip")
    cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off",
           "-fno-fast-math", "-I" + os.path.join(REPO, "include"), "-I" + os.path.join(PKG, "host"),
           "-I" + os.path.join(PKG, "csrc"), "--offload-device-only", "-S", "-o", "/tmp/spill_map.s",
           src] + sys.argv[2:]
    subprocess.run(cmd, check=True, capture_output=True)
    s = open("/tmp/spill_map.s").read()
    start = s.index(key)
    start = s.index(":", s.index("\n" + s[start:].split(":")[0].split("\n")[-1], start - 200))
    lines = s[start:s.index(".Lfunc_end", start)].splitlines()
    lab = {}
    for i, l in enumerate(lines):
        m = re.match(r"^(\.LBB\w+):", l)
        if m:
            lab[m.group(1)] = i
    loops = []
    for i, l in enumerate(lines):
        m = re.search(r"s_c?branch\w* (\.LBB\w+)", l)
        if m and m.group(1) in lab and lab[m.group(1)] < i:
            loops.append((lab[m.group(1)], i))
    for i, l in enumerate(lines):
        if "scratch_" in l:
            inl = [lp for lp in loops if lp[0] <= i <= lp[1]]
            inner = min(inl, key=lambda x: x[1] - x[0]) if inl else None
            print(i, l.strip()[:70], "| depth", len(inl), "inner", inner)


if __name__ == "__main__":
    main()
