#!/bin/bash
# GPU-box session for the candidate-list work: the exactness tests, a
# kernel-trace profile of the C5 bench (per-kernel list timings), and C5 bench
# lines at a few camera slacks.  Each GPU step has its own time limit; the
# first crash or timeout ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-lists}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread \
    -k "${PYTEST_K:-exact or c5 or synthetic or zero_normal or golden}" > "$OUT/pytest.log" 2>&1
rc=$?; tail -3 "$OUT/pytest.log"; echo "pytest rc=$rc"
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv \
    -- python3 bench.py --no-cpu --steps 5 --warmup 1 > "$OUT/trace.log" 2>&1 || exit $?
echo traced
for e in ${SLACKS:-64}; do
  timeout -k 10 200 python bench.py --no-cpu --steps 10 --warmup 2 --camera-slack $e \
      > "$OUT/cs_$e.json" 2> "$OUT/cs_$e.err" || exit $?
  echo "slack $e done"
done
