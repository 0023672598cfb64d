#!/bin/bash
# GPU suite of the default build, then an A/B of library variants on a
# workload (tools/ab_bench.sh): one gpurun call.
#   VARIANTS="nopf" WL=c5 gpurun --timeout 900 -- bash tools/gpu_ab.sh <tag> [pytest -k expr]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; export TMPDIR=/tmp
T=${1:?tag}; O=gpurun_out/$T; mkdir -p $O
K=${2:-}
if [ "${SUITE:-1}" = 1 ]; then
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ${K:+-k "$K"} > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
  tail -1 $O/pytest.log
fi
timeout -k 10 600 bash tools/ab_bench.sh > $O/ab.log 2>&1 || { tail -20 $O/ab.log; exit 1; }
cat $O/ab.log
