#!/bin/bash
# C5 frame time vs device octree build parameters (RT_DEV_LEAF leaf cap,
# RT_DEV_CLIP clip level), bench.py render-kernel and list times.
#   CFGS="leaf:clip ..." bash tools/build_sweep.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/bsweep
for cfg in ${CFGS:-12:7}; do
  RT_DEV_LEAF=${cfg%%:*} RT_DEV_CLIP=${cfg##*:} timeout -k 10 200 python3 bench.py --no-cpu --steps 8 \
      --warmup 2 > gpurun_out/bsweep/$cfg.json 2> gpurun_out/bsweep/$cfg.err || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/bsweep/$cfg.json')); r=d['roofline']; c=d['config']['accel_build']; print('$cfg', 'frame', d['ms_per_step'], 'kernel', r['kernel_ms'], 'lists', r['candidate_lists_ms'], 'nodes', c['nodes'], 'recs', c['records'], 'sh_nodes', r['per_lane']['shadow_nodes_per_query'], 'sh_tris', r['per_lane']['shadow_tris_per_query'])"
done
