set -u
# light buffers with inline records: shadow tests, then A/B of the query's
# prefetch / shade occupancy variants on C5
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r03t
timeout -k 10 400 python -u -m pytest tests/test_gpu.py -x -q --timeout 300 --timeout-method thread -k "shadow or light_buffer or no_camera or golden" > gpurun_out/r03t/pytest.log 2>&1 || { tail -40 gpurun_out/r03t/pytest.log; exit 1; }
tail -2 gpurun_out/r03t/pytest.log
VARIANTS="nopf pf6" WL=c5 bash tools/ab_bench.sh > gpurun_out/r03t/ab.log 2>&1 || { cat gpurun_out/r03t/ab.log; exit 1; }
cat gpurun_out/r03t/ab.log
for v in default nopf pf6; do python3 -c "import json; d=json.load(open('gpurun_out/ab/${v}_2.json')); r=d['roofline']; print('$v', {k: v['ms'] for k, v in r['kernels'].items()})"; done
