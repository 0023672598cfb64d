#!/bin/bash
# One rocprofv3 PMC pass over a short bench run (counters only, no tracing
# domains), reduced to per-launch averages of each uninstrumented render
# kernel (trace_kernel, shade_kernel, fold_kernel; the "<..., false, ...>"
# instantiations), written as {kernel: {counter: per-launch value}}.
#   tools/pmc_pass.sh <outdir> "<counters>" [bench args...]
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=$1; shift
ctr=$1; shift
timeout -s KILL 300 rocprofv3 --pmc $ctr -d "$out" -o pmc --output-format csv \
    -- python3 bench.py --no-cpu --steps 2 --warmup 0 "$@" > "$out.log" 2>&1
python3 tools/pmc_reduce.py "$out" -o "$out.json"
