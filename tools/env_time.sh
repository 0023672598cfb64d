#!/bin/bash
# Render-kernel time (bench.py, HIP events) per tuning configuration.
#   tools/env_time.sh "<cfg> <cfg> ..." "<workloads>"
# cfg = comma-separated VAR=value list applied to the library's tuning knobs
# (RT_TRAV, RT_PACKET_MIN, RT_MIN_WAVES, RT_OCT_C_BOX, RT_OCT_LEAF_CAP, ...);
# "-" = defaults.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for cfg in $1; do
  for wl in $2; do
    envs=()
    [ "$cfg" != "-" ] && IFS=',' read -ra envs <<< "$cfg"
    env "${envs[@]}" timeout -k 10 300 python3 bench.py --no-cpu --steps ${STEPS:-3} --workload $wl ${BENCH_EXTRA:-} \
        > gpurun_out/et.json 2> gpurun_out/et.err
    python3 -c "import json; d=json.load(open('gpurun_out/et.json')); r=d['roofline']; print('$cfg', '$wl', 'kernel_ms', r['kernel_ms'], 'Mrays', d['value'], 'nodes/q', r['node_fetches_per_query'], 'tris/q', r['tri_fetches_per_query'])"
  done
done
