set -u
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r03h
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03h/pytest.log 2>&1 || { tail -30 gpurun_out/r03h/pytest.log; exit 1; }
tail -3 gpurun_out/r03h/pytest.log
VARIANTS="nostream sw6 sw7" WL=c5 bash tools/ab_bench.sh > gpurun_out/r03h/ab.log 2>&1 || { cat gpurun_out/r03h/ab.log; exit 1; }
cat gpurun_out/r03h/ab.log
timeout -k 10 300 python -u tools/rank_share.py --nranks 1 8 --all-ranks --steps 5 --out gpurun_out/r03h/rank_share.json > gpurun_out/r03h/rank_share.log 2>&1 || exit 1
python3 -c "
import json; r=json.load(open('gpurun_out/r03h/rank_share.json'))
for n in (1,8):
  x=[e for e in r if e['nranks']==n]; print(n, 'max frame', max(e['frame_ms'] for e in x), 'max trace', max(e['trace_ms'] for e in x), 'max shade', max(e['shade_ms'] for e in x))"
