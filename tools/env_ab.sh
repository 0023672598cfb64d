#!/bin/bash
# A/B of an environment switch on one workload: bench.py frame and kernel
# times with and without ENV_B (e.g. ENV_B="RT_LISTS_SERIAL=1"), twice each,
# interleaved.  TAG=... ENV_B=... WL=c5 bash tools/env_ab.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-env_ab}
mkdir -p "$OUT"
WL=${WL:-c5}
for rep in 1 2; do
  for v in a b; do
    if [ $v = a ]; then e=""; else e="$ENV_B"; fi
    env $e timeout -k 10 200 python3 bench.py --no-cpu --steps 10 --warmup 2 --workload $WL \
        ${BENCH_EXTRA:-} > $OUT/${v}_$rep.json 2> $OUT/${v}_$rep.err || exit $?
    python3 -c "import json; d=json.load(open('$OUT/${v}_$rep.json')); r=d['roofline']; print('$v' if '$v'=='a' else '$ENV_B', $rep, 'frame_ms', d['ms_per_step'], 'kernel_ms', r['kernel_ms'], 'lists_ms', r['candidate_lists_ms'], 'Mrays', d['value'])"
  done
done
