set -u
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r03i
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -x -q --timeout 200 --timeout-method thread -k "shadow or light_buffer" > gpurun_out/r03i/pytest_lb.log 2>&1 || { tail -40 gpurun_out/r03i/pytest_lb.log; exit 1; }
tail -3 gpurun_out/r03i/pytest_lb.log
timeout -k 10 300 python3 -u bench.py --no-cpu --steps 10 --warmup 2 > gpurun_out/r03i/bench.json 2> gpurun_out/r03i/bench.err || { tail -20 gpurun_out/r03i/bench.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/r03i/bench.json')); r=d['roofline']
print('frame', d['ms_per_step'], 'Mrays', d['value'], {k: v['ms'] for k, v in r['kernels'].items()}, 'lists', r['candidate_lists_ms'], 'build', d['config'].get('accel_build'))
print('shadow per lane', r['per_lane'])"
timeout -k 10 300 python -u tools/c5_shadow.py --stride 16 --tag r03i > gpurun_out/r03i/c5_shadow.log 2>&1 || { tail -20 gpurun_out/r03i/c5_shadow.log; exit 1; }
tail -2 gpurun_out/r03i/c5_shadow.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03i/pytest.log 2>&1 || { tail -40 gpurun_out/r03i/pytest.log; exit 1; }
tail -3 gpurun_out/r03i/pytest.log
