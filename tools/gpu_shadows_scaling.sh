#!/bin/bash
# Every shadow query of the C5 frame against brute force (proven mode,
# tools/c5_shadow.py, ~5 min) and the per-rank cost of 1/2/4/8-way splits on
# one GPU with and without the triangle-parallel lists (tools/rank_share.py).
#   gpurun --timeout 1200 -- bash tools/gpu_shadows_scaling.sh <tag>
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; export TMPDIR=/tmp
T=${1:?tag}; O=gpurun_out/${T}_c5; mkdir -p $O
timeout -k 10 550 python3 -u tools/c5_shadow.py --all --stride 16 --exact 1 --tag ${T}_e1 > gpurun_out/c5_shadow_${T}_e1.log 2>&1 || { tail -5 gpurun_out/c5_shadow_${T}_e1.log; exit 1; }
tail -1 gpurun_out/c5_shadow_${T}_e1.log | cut -c1-300
timeout -k 10 500 python3 tools/rank_share.py --nranks 1 2 4 8 --all-ranks --partition --steps 3 --out $O/rank_share.json > $O/rank_share.log 2>&1 || { tail -20 $O/rank_share.log; exit 1; }
grep '"nranks": 8' $O/rank_share.log | cut -c1-200
