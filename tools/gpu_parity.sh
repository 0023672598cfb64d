#!/bin/bash
# Whole-frame C5 parity, one quarter per gpurun call (~9 min each): every
# tile of ranks [64 q, 64 q + 63] of a 256-way split rendered with the
# shipped defaults and by brute force (tools/c5_exact.py), compared bit for
# bit; parts 0-3 cover the frame.  Merge: tools/c5_exact_summary.py.
#   gpurun --timeout 1200 -- bash tools/gpu_parity.sh <tag> <q>
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; export TMPDIR=/tmp; mkdir -p gpurun_out
T=${1:?tag}; Q=${2:?quarter 0-3}
R0=$((64 * Q)); R1=$((R0 + 63)); L=gpurun_out/c5_exact_${T}_$Q.log
timeout -k 10 1100 python3 -u tools/c5_exact.py --grid 32 --tris 9776 --W 3840 --H 2160 --nranks 256 \
    --ranks $R0-$R1 --tag ${T}_$Q > $L 2>&1 || { tail -5 $L; exit 1; }
tail -2 $L | cut -c1-300
