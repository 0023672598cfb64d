#!/bin/bash
# GPU suite + per-rank scaling of a tree (one gpurun call, ~6 min): pytest -m
# gpu, smoke(), the default C5 bench line, the per-rank cost of 1/2/4/8-way
# splits (tools/rank_share.py, with the triangle-parallel lists) and the
# per-tile cost map at N = 1 (tools/tile_cost.py --npy, for tools/tile_map_sim.py).
#   gpurun --timeout 1200 -- bash tools/gpu_suite_scaling.sh <tag>
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; export TMPDIR=/tmp
T=${1:?tag}; O=gpurun_out/$T; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
timeout -k 10 200 python3 bench.py --steps 10 --warmup 2 > $O/bench_c5.json 2> $O/bench_c5.err || { tail -20 $O/bench_c5.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_c5.json')); r=d['roofline']; print('C5', d['ms_per_step'], 'ms', d['value'], 'Mrays/s; trace', r['kernels']['trace']['ms'], 'shade', r['kernels']['shade']['ms'], 'lists', r['candidate_lists_ms'])"
[ "${SCALING:-1}" = 1 ] || exit 0
timeout -k 10 500 python3 tools/rank_share.py --nranks 1 2 4 8 --all-ranks --partition --steps 3 --out $O/rank_share.json > $O/rank_share.log 2>&1 || { tail -20 $O/rank_share.log; exit 1; }
python3 tools/rank_share_summary.py $O/rank_share.json
timeout -k 10 200 python3 -u tools/tile_cost.py --synthetic 32 --W 3840 --H 2160 --npy $O/tile_cost_n1.npz --out $O/tile_cost_n1.json > $O/tile_cost.log 2>&1 || { tail -5 $O/tile_cost.log; exit 1; }
echo done
