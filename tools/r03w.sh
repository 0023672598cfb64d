set -u
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r03w
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03w/pytest.log 2>&1 || { tail -40 gpurun_out/r03w/pytest.log; exit 1; }
tail -2 gpurun_out/r03w/pytest.log
TAG=r03w_c5 bash tools/gpu_profile.sh > gpurun_out/r03w/profile.log 2>&1 || { tail -30 gpurun_out/r03w/profile.log; exit 1; }
tail -3 gpurun_out/r03w/profile.log | cut -c1-600
timeout -k 10 400 python -u tools/rank_share.py --nranks 1 2 4 8 --all-ranks --steps 5 --out gpurun_out/r03w/rank_share.json > gpurun_out/r03w/rank_share.log 2>&1 || exit 1
python3 -c "
import json; r=json.load(open('gpurun_out/r03w/rank_share.json'))
for n in (1,2,4,8):
  x=[e for e in r if e['nranks']==n]; print(n, 'max frame', max(e['frame_ms'] for e in x), 'min', min(e['frame_ms'] for e in x), 'lists', max(e['lists_ms'] for e in x), 'trace', max(e['trace_ms'] for e in x), 'shade', max(e['shade_ms'] for e in x), 'wall', max(e['wall_ms_per_frame'] for e in x))"
