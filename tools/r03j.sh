set -u
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r03j
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -x -q --timeout 200 --timeout-method thread -k "shadow or light_buffer" > gpurun_out/r03j/pytest_lb.log 2>&1 || { tail -40 gpurun_out/r03j/pytest_lb.log; exit 1; }
tail -2 gpurun_out/r03j/pytest_lb.log
VARIANTS="bbox" WL=c5 bash tools/ab_bench.sh > gpurun_out/r03j/ab.log 2>&1 || { cat gpurun_out/r03j/ab.log; exit 1; }
cat gpurun_out/r03j/ab.log
python3 -c "
import json; d=json.load(open('gpurun_out/ab/default_1.json')); r=d['roofline']
print({k: v['ms'] for k, v in r['kernels'].items()}, d['config']['accel_build'], r['per_lane'])"
timeout -k 10 400 python -u tools/rank_share.py --nranks 1 2 4 8 --all-ranks --steps 5 --out gpurun_out/r03j/rank_share.json > gpurun_out/r03j/rank_share.log 2>&1 || exit 1
python3 -c "
import json; r=json.load(open('gpurun_out/r03j/rank_share.json'))
for n in (1,2,4,8):
  x=[e for e in r if e['nranks']==n]; print(n, 'max frame', max(e['frame_ms'] for e in x), 'lists', max(e['lists_ms'] for e in x), 'trace', max(e['trace_ms'] for e in x), 'shade', max(e['shade_ms'] for e in x))"
