#!/usr/bin/env python3
"""Per-kernel register / scratch / occupancy summary of a HIP source file,
from the compiler's kernel-resource-usage remarks (no GPU needed).

    python tools/kres.py [raytracing-gpu_amd/csrc/rt_render.hip] [-D...]
"""
import os
import re
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "raytracing-gpu_amd")


def main():
    src = sys.argv[1] if len(sys.argv) > 1 else os.path.join(PKG, "csrc", "rt_render.hip")
    extra = sys.argv[2:]
    cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC",
           "-ffp-contract=off", "-fno-fast-math", "-I" + os.path.join(REPO, "include"),
           "-I" + os.path.join(PKG, "host"), "-I" + os.path.join(PKG, "csrc"), "-c", src,
           "-o", "/tmp/kres.o", "--offload-device-only", "-Rpass-analysis=kernel-resource-usage"] + extra
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode:
        sys.stderr.write(r.stderr)
        sys.exit(r.returncode)
    rows, cur = [], None
    for line in r.stderr.splitlines():
        m = re.search(r"remark: +(.*?): (.*?) \[-Rpass", line)
        if not m:
            continue
        k, v = m.group(1).strip(), m.group(2).strip()
        if k == "Function Name":
            cur = {"name": v}
            rows.append(cur)
        elif cur is not None:
            cur[k] = v
    keys = ["VGPRs", "AGPRs", "SGPRs", "ScratchSize [bytes/lane]", "Occupancy [waves/SIMD]",
            "SGPRs Spill", "VGPRs Spill", "LDS Size [bytes/block]"]
    print("%-60s %s" % ("kernel", " ".join("%8s" % k.split()[0][:8] for k in keys)))
    for row in rows:
        name = subprocess.run(["c++filt", row["name"]], capture_output=True, text=True).stdout.strip()
        print("%-60s %s" % (name[:60], " ".join("%8s" % row.get(k, "-") for k in keys)))


if __name__ == "__main__":
    main()
