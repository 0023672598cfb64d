set -u
# early SAFE / AWAY exits in the lists' float fast path: the list tests,
# the C5 bench, per-rank cost at N = 1, 2, 4, 8
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r03s
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03s/pytest.log 2>&1 || { tail -40 gpurun_out/r03s/pytest.log; exit 1; }
tail -2 gpurun_out/r03s/pytest.log
timeout -k 10 200 python3 bench.py --no-cpu --steps 10 --warmup 2 > gpurun_out/r03s/bench.json 2> gpurun_out/r03s/bench.err || { tail -5 gpurun_out/r03s/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r03s/bench.json')); r=d['roofline']; print('c5', d['ms_per_step'], {k: v['ms'] for k, v in r['kernels'].items()}, r['candidate_lists_ms'])"
timeout -k 10 400 python -u tools/rank_share.py --nranks 1 2 4 8 --all-ranks --steps 5 --out gpurun_out/r03s/rank_share.json > gpurun_out/r03s/rank_share.log 2>&1 || exit 1
python3 -c "
import json; r=json.load(open('gpurun_out/r03s/rank_share.json'))
for n in (1,2,4,8):
  x=[e for e in r if e['nranks']==n]; print(n, 'max frame', max(e['frame_ms'] for e in x), 'lists', max(e['lists_ms'] for e in x), 'trace', max(e['trace_ms'] for e in x), 'shade', max(e['shade_ms'] for e in x))"
