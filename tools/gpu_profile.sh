#!/bin/bash
# GPU-box profiling session for one bench workload: the bench line, a
# rocprofv3 kernel-trace/stats pass, and two PMC passes (FETCH_SIZE,
# WRITE_SIZE; separate runs, no tracing domains) reduced by pmc_traffic.py.
# Every GPU step has its own time limit; the first failure ends the script.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
WL=${WL:-c5}
TAG=${TAG:-r01_$WL}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
B="bench.py --workload $WL"
echo "== bench $WL"
timeout -k 10 ${BENCH_TIMEOUT:-400} python3 $B --steps ${STEPS:-5} --warmup 1 \
    > "$OUT/bench.json" 2> "$OUT/bench.err"
cat "$OUT/bench.json"
echo "== kernel trace"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv \
    -- python3 $B --no-cpu --steps 5 --warmup 1 > "$OUT/trace.log" 2>&1
echo "== pmc FETCH_SIZE"
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE -d "$OUT/pmc_fetch" -o fetch --output-format csv \
    -- python3 $B --no-cpu --steps 2 --warmup 0 > "$OUT/pmc_fetch.log" 2>&1
echo "== pmc WRITE_SIZE"
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE -d "$OUT/pmc_write" -o write --output-format csv \
    -- python3 $B --no-cpu --steps 2 --warmup 0 > "$OUT/pmc_write.log" 2>&1
python3 tools/pmc_traffic.py "$OUT/pmc_fetch" "$OUT/pmc_write" -o "$OUT/traffic.json"
if [ -n "${EXTRA:-}" ]; then
  echo "== extra"
  timeout -k 10 ${EXTRA_TIMEOUT:-400} bash -c "$EXTRA" > "$OUT/extra.log" 2>&1
  tail -30 "$OUT/extra.log"
fi
echo "done"
