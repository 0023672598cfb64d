set -u
# exact-shadow mode with deferred off-box queries: GPU suite, C5 A/B,
# every C5 shadow query of the frame vs brute force in both modes
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r03p
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03p/pytest.log 2>&1 || { tail -40 gpurun_out/r03p/pytest.log; exit 1; }
tail -2 gpurun_out/r03p/pytest.log
for x in 0 1; do
  timeout -k 10 200 python3 bench.py --no-cpu --steps 10 --warmup 2 --exact-shadows $x > gpurun_out/r03p/bench_exact$x.json 2> gpurun_out/r03p/bench_exact$x.err || { tail -5 gpurun_out/r03p/bench_exact$x.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r03p/bench_exact$x.json')); r=d['roofline']; print('exact $x', d['ms_per_step'], {k: v['ms'] for k, v in r['kernels'].items()}, r['candidate_lists_ms'], d['config']['accel_build'], r['per_lane'])"
done
for x in 1 0; do
  timeout -k 10 400 python -u tools/c5_shadow.py --stride 1 --exact $x --probe 4000 --tag r03p_e$x > gpurun_out/r03p/c5_shadow_e$x.log 2>&1 || { tail -5 gpurun_out/r03p/c5_shadow_e$x.log; exit 1; }
  cut -c1-1200 gpurun_out/r03p/c5_shadow_e$x.log
done
