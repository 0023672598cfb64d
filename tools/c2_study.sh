#!/bin/bash
# C2 (spheres.svati 1920x1080) under each acceleration: bench line (per-lane
# work counters, render-kernel time) and one SQ VALU PMC pass per variant.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/c2_study
mkdir -p $OUT
for acc in ${ACCELS:-flat octree octree_gpu}; do
  echo "== $acc"
  timeout -k 10 300 python3 bench.py --workload c2 --accel $acc --no-cpu --steps 3 --warmup 1 \
      > $OUT/bench_$acc.json 2> $OUT/bench_$acc.err
  bash tools/pmc_pass.sh $OUT/pmc_$acc \
      "SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAVES GRBM_GUI_ACTIVE" \
      --workload c2 --accel $acc > /dev/null
done
echo done
