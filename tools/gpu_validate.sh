#!/bin/bash
# GPU-box validation of a tree (one gpurun call, ~4 min): the GPU suite,
# smoke(), the default C5 bench line (with its CPU baseline), the C1-C4 lines
# (tools/bench_all.sh) and the C5 profile (tools/gpu_profile.sh) under
# gpurun_out/$TAG_val and gpurun_out/$TAG_c5.  Each GPU step has its own
# time limit; the first failure ends the script.
#   gpurun --timeout 1200 -- bash tools/gpu_validate.sh <tag>
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; export TMPDIR=/tmp
T=${1:?tag}; O=gpurun_out/${T}_val; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 200 python3 bench.py > $O/bench_c5.json 2> $O/bench_c5.err || { tail -20 $O/bench_c5.err; exit 1; }
TAG=${T}_val/all timeout -k 10 900 bash tools/bench_all.sh || exit 1
TAG=${T}_c5 timeout -k 10 1200 bash tools/gpu_profile.sh > $O/profile.log 2>&1 || { tail -20 $O/profile.log; exit 1; }
tail -3 $O/profile.log
