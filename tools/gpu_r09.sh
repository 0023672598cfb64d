#!/bin/bash
# Round 6 GPU session: GPU suite (optional -k), then C5 bench lines.
# Every GPU step has its own time limit; a crash or timeout stops the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r09}
mkdir -p $OUT
if [ -z "${NO_TESTS:-}" ]; then
  timeout -k 10 ${PYTEST_TIMEOUT:-420} python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    ${PYTEST_K:+-k "$PYTEST_K"} > $OUT/pytest.log 2>&1
  rc=$?
  tail -4 $OUT/pytest.log
  echo "pytest rc=$rc"
  if [ $rc -gt 1 ]; then exit $rc; fi
fi
i=0
for args in ${BENCHES:-"--steps 20 --warmup 3 --no-cpu"}; do :; done
IFS=';' read -ra BL <<< "${BENCHES:---steps 20 --warmup 3 --no-cpu}"
for args in "${BL[@]}"; do
  i=$((i+1))
  timeout -k 10 ${BENCH_TIMEOUT:-300} python bench.py $args > $OUT/bench$i.json 2> $OUT/bench$i.err
  rc=$?
  echo "bench$i ($args) rc=$rc"
  tail -2 $OUT/bench$i.err
  python3 -c "import json,sys;d=json.load(open('$OUT/bench$i.json'));print({k:d[k] for k in ('value','ms_per_step','ms_per_step_fresh')}, d['roofline']['kernels']['trace']['ms'], d['roofline']['kernels']['shade']['ms'], d['roofline']['candidate_lists_ms'], d.get('fresh_camera'))" || true
  if [ $rc -ne 0 ]; then exit $rc; fi
done
