#!/bin/bash
# Kernel trace of the produce step (tools/prof_produce.py) -> per-call
# timeline of one rank-0 and one rank-7 produce (tools/produce_timeline.py).
#   gpurun --timeout 600 -- bash tools/gpu_produce_trace.sh <tag>
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; export TMPDIR=/tmp
T=${1:?tag}; O=gpurun_out/$T; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prod -o prod --output-format csv \
    -- python3 tools/prof_produce.py --n ${N:-8} --steps 20 --consume > $O/prod.log 2>&1 || { tail -20 $O/prod.log; exit 1; }
grep produce_ms $O/prod.log
python3 tools/produce_timeline.py $O/prod/prod_kernel_trace.csv --n ${N:-8} --steps 20
