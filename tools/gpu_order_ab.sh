#!/bin/bash
# Per-rank trace cost at N = 8 (and the C5 bench at N = 1) for the default
# library and the variants named in VARIANTS (raytracing-gpu_amd/lib/var_<v>):
# one gpurun call.
#   VARIANTS="nocost" gpurun --timeout 900 -- bash tools/gpu_order_ab.sh <tag>
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; export TMPDIR=/tmp
T=${1:?tag}; O=gpurun_out/$T; mkdir -p $O
if [ "${SUITE:-1}" = 1 ]; then
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ${K:+-k "$K"} > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
  tail -1 $O/pytest.log
fi
for v in default ${VARIANTS:-}; do
  lib=raytracing-gpu_amd/lib/librtgpu.so
  [ $v = default ] || lib=raytracing-gpu_amd/lib/var_$v/librtgpu.so
  RTGPU_LIB=$lib timeout -k 10 300 python3 tools/rank_share.py --nranks ${NR:-8} --all-ranks --steps 5 \
      --out $O/rs_$v.json > $O/rs_$v.log 2>&1 || { tail -20 $O/rs_$v.log; exit 1; }
  RTGPU_LIB=$lib timeout -k 10 200 python3 bench.py --no-cpu --steps 10 --warmup 2 > $O/bench_$v.json 2> $O/bench_$v.err \
      || { tail -20 $O/bench_$v.err; exit 1; }
  python3 - $O/rs_$v.json $O/bench_$v.json $v <<'PY'
import json, sys
rs = json.load(open(sys.argv[1])); b = json.load(open(sys.argv[2]))
tr = [r["trace_ms"] for r in rs]; sh = [r["shade_ms"] for r in rs]; fr = [r["frame_ms"] for r in rs]
print(sys.argv[3], "N8 trace", tr, "max/mean %.3f" % (max(tr) / (sum(tr) / len(tr))), "slowest frame", max(fr),
      "| C5", b["ms_per_step"], "trace", b["roofline"]["kernels"]["trace"]["ms"])
PY
done
echo done
