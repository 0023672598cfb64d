set -u
# proven light buffers: GPU suite, C5 A/B (slack vs proven), C5 shadow checks
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r03n
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03n/pytest.log 2>&1 || { tail -40 gpurun_out/r03n/pytest.log; exit 1; }
tail -2 gpurun_out/r03n/pytest.log
for x in 0 1; do
  timeout -k 10 200 python3 bench.py --no-cpu --steps 10 --warmup 2 --exact-shadows $x > gpurun_out/r03n/bench_exact$x.json 2> gpurun_out/r03n/bench_exact$x.err || { tail -5 gpurun_out/r03n/bench_exact$x.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r03n/bench_exact$x.json')); r=d['roofline']; print('exact $x', d['ms_per_step'], {k: v['ms'] for k, v in r['kernels'].items()}, r['candidate_lists_ms'], d['config']['accel_build'], r['per_lane'])"
done
for x in 1 0; do
  timeout -k 10 300 python -u tools/c5_shadow.py --stride 16 --exact $x --probe 2000 --tag r03n_e$x > gpurun_out/r03n/c5_shadow_e$x.log 2>&1 || { tail -5 gpurun_out/r03n/c5_shadow_e$x.log; exit 1; }
  cut -c1-1500 gpurun_out/r03n/c5_shadow_e$x.log
done
# camera-slack sweep (the lists adapt: exact at every slack)
for cs in 32 96 128 192; do
  timeout -k 10 200 python3 bench.py --no-cpu --steps 10 --warmup 2 --camera-slack $cs > gpurun_out/r03n/bench_cs$cs.json 2> gpurun_out/r03n/bench_cs$cs.err || { tail -5 gpurun_out/r03n/bench_cs$cs.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r03n/bench_cs$cs.json')); r=d['roofline']; print('camera slack $cs', d['ms_per_step'], {k: v['ms'] for k, v in r['kernels'].items()}, r['candidate_lists_ms'], r['candidate_entries'])"
done
