set -u
# C5 profile of the final tree (kernel trace, HBM traffic, SQ passes, bench) and the per-rank split
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r04q; export TMPDIR=/tmp
TAG=r04q_c5 bash tools/gpu_profile.sh > gpurun_out/r04q/profile.log 2>&1 || { tail -30 gpurun_out/r04q/profile.log; exit 1; }
tail -3 gpurun_out/r04q/profile.log | cut -c1-400
timeout -k 10 400 python -u tools/rank_share.py --nranks 1 2 4 8 --all-ranks --steps 5 --out gpurun_out/r04q/rank_share.json > gpurun_out/r04q/rank_share.log 2>&1 || { tail -5 gpurun_out/r04q/rank_share.log; exit 1; }
python3 -c "
import json; r=json.load(open('gpurun_out/r04q/rank_share.json'))
for n in (1,2,4,8):
  x=[e for e in r if e['nranks']==n]; print(n, 'max frame', max(e['frame_ms'] for e in x), 'min', min(e['frame_ms'] for e in x), 'lists', max(e['lists_ms'] for e in x), 'trace', max(e['trace_ms'] for e in x), 'shade', max(e['shade_ms'] for e in x), 'wall', max(e['wall_ms_per_frame'] for e in x))"
