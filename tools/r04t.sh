set -u
# final tree: C5 profile (kernel trace, HBM traffic, SQ passes, bench), per-rank split, C1-C4 bench lines
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r04t; export TMPDIR=/tmp
TAG=r04t_c5 bash tools/gpu_profile.sh > gpurun_out/r04t/profile.log 2>&1 || { tail -30 gpurun_out/r04t/profile.log; exit 1; }
tail -3 gpurun_out/r04t/profile.log | cut -c1-300
timeout -k 10 400 python -u tools/rank_share.py --nranks 1 2 4 8 --all-ranks --steps 5 --out gpurun_out/r04t/rank_share.json > gpurun_out/r04t/rank_share.log 2>&1 || { tail -5 gpurun_out/r04t/rank_share.log; exit 1; }
python3 -c "
import json; r=json.load(open('gpurun_out/r04t/rank_share.json'))
for n in (1,2,4,8):
  x=[e for e in r if e['nranks']==n]; print(n, 'max frame', max(e['frame_ms'] for e in x), 'min', min(e['frame_ms'] for e in x), 'lists', max(e['lists_ms'] for e in x), 'trace', max(e['trace_ms'] for e in x), 'shade', max(e['shade_ms'] for e in x), 'wall', max(e['wall_ms_per_frame'] for e in x))"
for wl in c1 c2 c3 c4; do
  timeout -k 10 300 python3 bench.py --workload $wl --steps 10 --warmup 2 --cpu-seconds 12 > gpurun_out/r04t/bench_$wl.json 2> gpurun_out/r04t/bench_$wl.err || { tail -5 gpurun_out/r04t/bench_$wl.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r04t/bench_$wl.json')); r=d['roofline']; print('$wl', d['value'], d['ms_per_step'], {k: v['ms'] for k, v in r['kernels'].items()}, r.get('candidate_lists_ms'), (d.get('cpu_baseline') or {}).get('value'))"
done
