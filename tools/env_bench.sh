#!/bin/bash
# A/B of a context-creation env knob: one bench line per value.
# usage: KNOB=RT_ENTRY_DEPTH VALUES="0 4 8" TAG=x ARGS="--steps 20 --warmup 3 --no-cpu --camera-pan 0" tools/env_bench.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-envab}
mkdir -p $OUT
for v in $VALUES; do
  env $KNOB=$v timeout -k 10 ${BENCH_TIMEOUT:-240} python bench.py $ARGS > $OUT/$KNOB-$v.json 2> $OUT/$KNOB-$v.err
  rc=$?
  echo "$KNOB=$v rc=$rc"
  python3 -c "import json;d=json.load(open('$OUT/$KNOB-$v.json'));r=d['roofline'];print(d['ms_per_step'], r['kernels']['trace']['ms'], r['kernels']['shade']['ms'], r['candidate_lists_ms'], r['closest_fetches_per_query'], r['per_lane']['closest_nodes_per_query'], 'fresh', d.get('ms_per_step_fresh'), (d.get('fresh_camera') or {}).get('candidate_lists_ms'))" || true
  if [ $rc -ne 0 ]; then exit $rc; fi
done
