#!/bin/bash
# Partition-list and bench A/B of the default library against variants
# (raytracing-gpu_amd/lib/var_<v>): rank_share at N = 1 / 4 / 8 with the
# triangle-parallel lists, and the C5 bench, per library.  One gpurun call.
#   VARIANTS="v1 v2" KSEL="pytest -k expr" gpurun -- bash tools/gpu_lib_ab.sh <tag>
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; export TMPDIR=/tmp
T=${1:?tag}; O=gpurun_out/$T; mkdir -p $O
if [ -n "${KSEL:-}" ]; then
  timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "$KSEL" \
      > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
  tail -1 $O/pytest.log
fi
for v in default ${VARIANTS:-}; do
  lib=raytracing-gpu_amd/lib/librtgpu.so
  [ $v = default ] || lib=raytracing-gpu_amd/lib/var_$v/librtgpu.so
  RTGPU_LIB=$lib timeout -k 10 300 python3 tools/rank_share.py --nranks 1 4 8 --partition --steps 5 \
      --out $O/rs_$v.json > $O/rs_$v.log 2>&1 || { tail -20 $O/rs_$v.log; exit 1; }
  RTGPU_LIB=$lib timeout -k 10 200 python3 bench.py --no-cpu --steps 10 --warmup 2 > $O/bench_$v.json \
      2> $O/bench_$v.err || { tail -20 $O/bench_$v.err; exit 1; }
  python3 - $O/rs_$v.json $O/bench_$v.json $v <<'PY'
import json, sys
rs = json.load(open(sys.argv[1])); b = json.load(open(sys.argv[2]))
out = []
for r in rs:
    p = r.get("partition", {})
    out.append(f"N{r['nranks']}r{r['rank']} lists {r['lists_ms']} render {r['render_ms']}"
               + (f" produce {p['produce_ms_max']} consume {p['consume_ms_est']} part {p['frame_ms_without_exchange']}" if p else ""))
print(sys.argv[3], "| C5", b["ms_per_step"], "lists", b["roofline"]["candidate_lists_ms"])
print("   " + "\n   ".join(out))
PY
done
echo done
