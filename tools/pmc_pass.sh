#!/bin/bash
# One rocprofv3 PMC pass over a short bench run (counters only, no tracing
# domains), reduced to per-launch averages of the uninstrumented render kernel.
#   tools/pmc_pass.sh <outdir> "<counters>" [bench args...]
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=$1; shift
ctr=$1; shift
timeout -s KILL 300 rocprofv3 --pmc $ctr -d "$out" -o pmc --output-format csv \
    -- python3 bench.py --no-cpu --steps 2 --warmup 0 "$@" > "$out.log" 2>&1
python3 - "$out" <<'PY'
import collections, csv, glob, json, os, sys
d = sys.argv[1]
acc = collections.defaultdict(float)
disp = set()
for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        if "render_kernel" not in r["Kernel_Name"] or "false" not in r["Kernel_Name"]:
            continue
        acc[r["Counter_Name"]] += float(r["Counter_Value"])
        disp.add(r["Dispatch_Id"])
res = {k: v / max(1, len(disp)) for k, v in sorted(acc.items())}
res["dispatches"] = len(disp)
json.dump(res, open(d + ".json", "w"), indent=1)
print(json.dumps(res))
PY
