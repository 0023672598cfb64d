#!/bin/bash
# GPU-box profiling session for one bench workload:
#   1. rocprofv3 --kernel-trace --stats of a short bench run,
#   2. PMC passes (each its own run, counters only): FETCH_SIZE, WRITE_SIZE,
#      and the SQ VALU counters,
#   3. the bench line itself, carrying the PMC-derived roofline.traffic and
#      valu blocks.
# Every GPU step has its own time limit; the first failure ends the script.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
WL=${WL:-c5}
TAG=${TAG:-r02_$WL}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
B="bench.py --workload $WL"
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
echo "== pmc VALU"
bash tools/pmc_pass.sh "$OUT/pmc_valu" \
    "SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAVES GRBM_GUI_ACTIVE" \
    --workload $WL
echo "== bench $WL"
timeout -k 10 ${BENCH_TIMEOUT:-400} python3 $B --steps ${STEPS:-5} --warmup 1 \
    --traffic-json "$OUT/traffic.json" --valu-json "$OUT/pmc_valu.json" \
    > "$OUT/bench.json" 2> "$OUT/bench.err"
cat "$OUT/bench.json"
if [ -n "${EXTRA:-}" ]; then
  echo "== extra"
  timeout -k 10 ${EXTRA_TIMEOUT:-400} bash -c "$EXTRA" > "$OUT/extra.log" 2>&1
  tail -30 "$OUT/extra.log"
fi
echo "done"
