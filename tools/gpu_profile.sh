#!/bin/bash
# GPU-box profiling session for one bench workload (the render's three
# kernels: trace_kernel, shade_kernel, fold_kernel):
#   1. rocprofv3 --kernel-trace --stats of a short bench run,
#   2. PMC passes, each its own run, counters only (MI355X_MICROARCH.md: one
#      pass holds at most 8 SQ, 4 TCC -- FETCH_SIZE takes 3, WRITE_SIZE 2 --
#      and 2 GRBM counters): FETCH_SIZE; WRITE_SIZE; SQ pass A (wave-cycle
#      breakdown + VALU); SQ pass B (instruction mix),
#   3. the bench line itself, carrying the PMC-derived roofline traffic and
#      the per-kernel SQ block.
# Every GPU step has its own time limit; the first failure ends the script.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
WL=${WL:-c5}
TAG=${TAG:-r03_$WL}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
# the device code these passes measure (bench.py reports a profile's counters
# only for the tree whose device_code_hash() matches)
python3 -c "import sys; sys.argv=['x']; sys.path.insert(0, '.'); import bench; print(bench.device_code_hash())" > "$OUT/device_hash.txt"
B="bench.py --workload $WL ${BENCH_EXTRA:-}"
echo "== kernel trace"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv \
    -- python3 $B --no-cpu --steps 5 --warmup 1 > "$OUT/trace.log" 2>&1
echo "== pmc FETCH_SIZE"
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d "$OUT/pmc_fetch" -o fetch --output-format csv \
    -- python3 $B --no-cpu --steps 2 --warmup 0 > "$OUT/pmc_fetch.log" 2>&1
echo "== pmc WRITE_SIZE"
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d "$OUT/pmc_write" -o write --output-format csv \
    -- python3 $B --no-cpu --steps 2 --warmup 0 > "$OUT/pmc_write.log" 2>&1
python3 tools/pmc_traffic.py "$OUT/pmc_fetch" "$OUT/pmc_write" -o "$OUT/traffic.json"
echo "== pmc SQ A"
bash tools/pmc_pass.sh "$OUT/pmc_sqa" \
    "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_THREAD_CYCLES_VALU GRBM_GUI_ACTIVE" \
    --workload $WL ${BENCH_EXTRA:-}
echo "== pmc SQ B"
bash tools/pmc_pass.sh "$OUT/pmc_sqb" \
    "SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_SALU SQ_WAVES SQ_INSTS_VMEM_WR SQ_BUSY_CYCLES" \
    --workload $WL ${BENCH_EXTRA:-}
python3 - "$OUT" <<'PY'
import json, sys
d = sys.argv[1]
a = json.load(open(d + "/pmc_sqa.json"))
b = json.load(open(d + "/pmc_sqb.json"))
for k, v in b.items():
    a.setdefault(k, {}).update({c: x for c, x in v.items() if c != "dispatches"})
json.dump(a, open(d + "/pmc_sq.json", "w"), indent=1)
PY
echo "== bench $WL"
timeout -k 10 ${BENCH_TIMEOUT:-400} python3 $B --steps ${STEPS:-5} --warmup 1 \
    --traffic-json "$OUT/traffic.json" --valu-json "$OUT/pmc_sq.json" \
    > "$OUT/bench.json" 2> "$OUT/bench.err"
cat "$OUT/bench.json"
echo "done"
