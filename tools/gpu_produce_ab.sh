#!/bin/bash
# Triangle-parallel lists A/B on one GPU box (one gpurun call): the list /
# partition GPU tests, then per-producer produce times and the per-rank list
# and partition cost at N = 1, 4, 8 for each RT_CAND_CHUNK_SHIFT value given
# ("" = the library's default).
#   gpurun --timeout 900 -- bash tools/gpu_produce_ab.sh <tag> "" 10
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; export TMPDIR=/tmp
T=${1:?tag}; shift; O=gpurun_out/$T; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
    -k "${KSEL:-triangle_parallel or exchange or consumed or async or cand or partition}" > $O/pytest.log 2>&1 \
    || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for v in "$@"; do
  tag=${v:-default}
  echo "== chunk shift $tag"
  RT_CAND_CHUNK_SHIFT=$v timeout -k 10 200 python3 tools/prof_produce.py --n 8 --steps 20 > $O/produce_$tag.log 2>&1 \
      || { tail -20 $O/produce_$tag.log; exit 1; }
  cat $O/produce_$tag.log
  RT_CAND_CHUNK_SHIFT=$v timeout -k 10 300 python3 tools/rank_share.py --nranks 1 4 8 --partition --steps 5 \
      --out $O/rank_share_$tag.json > $O/rank_share_$tag.log 2>&1 || { tail -20 $O/rank_share_$tag.log; exit 1; }
  python3 - $O/rank_share_$tag.json <<'PY'
import json, sys
for r in json.load(open(sys.argv[1])):
    p = r.get("partition", {})
    print(r["nranks"], r["rank"], "lists", r["lists_ms"], "render", r["render_ms"], "produce_max", p.get("produce_ms_max"),
          "consume", p.get("consume_ms_est"))
PY
done
echo done
