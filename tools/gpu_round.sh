#!/bin/bash
# One GPU-box session: parity tests, then a short bench.  Every GPU step has its
# own time limit; a crash/timeout (not a plain test failure) stops the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
PYTEST_ARGS=${PYTEST_ARGS:-"-m gpu -q"}
if [ -n "${PYTEST_K:-}" ]; then
  timeout -k 10 ${PYTEST_TIMEOUT:-900} python -m pytest tests $PYTEST_ARGS -k "$PYTEST_K" > gpurun_out/pytest_gpu.log 2>&1
else
  timeout -k 10 ${PYTEST_TIMEOUT:-900} python -m pytest tests $PYTEST_ARGS > gpurun_out/pytest_gpu.log 2>&1
fi
rc=$?
tail -5 gpurun_out/pytest_gpu.log
echo "pytest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
if [ -n "${EXTRA:-}" ]; then
  timeout -k 10 ${EXTRA_TIMEOUT:-600} bash -c "$EXTRA" > gpurun_out/extra.log 2>&1
  rc=$?
  tail -40 gpurun_out/extra.log
  echo "extra rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
fi
if [ -n "${BENCH_ARGS:-}" ]; then
  timeout -k 10 ${BENCH_TIMEOUT:-600} python bench.py $BENCH_ARGS > gpurun_out/bench.json 2> gpurun_out/bench.err
  rc=$?
  tail -3 gpurun_out/bench.err
  cat gpurun_out/bench.json
  echo "bench rc=$rc"
  exit $rc
fi
