#!/bin/bash
# Kernel time (bench, HIP events) and a VALU-utilisation PMC pass per
# traversal policy (env RT_TRAV).  tools/trav_cmp.sh "<policies>" [bench args]
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
pols=$1; shift
for tv in $pols; do
  RT_TRAV=$tv timeout -k 10 300 python3 bench.py --no-cpu --steps 3 "$@" > gpurun_out/tc_$tv.json 2>/dev/null
  python3 -c "import json; d=json.load(open('gpurun_out/tc_$tv.json')); r=d['roofline']; print('trav $tv', d['config']['workload'][:3], 'kernel_ms', r['kernel_ms'], 'Mrays', d['value'], 'nodes/q', r['node_visits_per_query'], 'tris/q', r['tri_tests_per_query'])"
  RT_TRAV=$tv bash tools/pmc_pass.sh gpurun_out/pmc_u_$tv "SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_VALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD" "$@"
done
