#!/bin/bash
# Render-kernel time (bench.py, HIP events) per traversal policy and workload.
#   tools/trav_time.sh "<RT_TRAV:RT_PACKET_MIN ...>" "<workloads>"
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for cfg in $1; do
  for wl in $2; do
    RT_TRAV=${cfg%%:*} RT_PACKET_MIN=${cfg##*:} timeout -k 10 300 python3 bench.py --no-cpu --steps 3 --workload $wl > gpurun_out/tt.json 2>/dev/null
    python3 -c "import json; d=json.load(open('gpurun_out/tt.json')); r=d['roofline']; print('$cfg', '$wl', 'kernel_ms', r['kernel_ms'], 'Mrays', d['value'])"
  done
done
