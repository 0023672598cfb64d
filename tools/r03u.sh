set -u
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r03u
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03u/pytest.log 2>&1 || { tail -40 gpurun_out/r03u/pytest.log; exit 1; }
tail -2 gpurun_out/r03u/pytest.log
for x in 0 1; do
  timeout -k 10 200 python3 bench.py --no-cpu --steps 10 --warmup 2 --exact-shadows $x > gpurun_out/r03u/bench_exact$x.json 2> gpurun_out/r03u/bench_exact$x.err || { tail -5 gpurun_out/r03u/bench_exact$x.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r03u/bench_exact$x.json')); r=d['roofline']; print('exact $x', d['ms_per_step'], d['value'], {k: v['ms'] for k, v in r['kernels'].items()}, r['candidate_lists_ms'])"
done
timeout -k 10 300 python -u tools/c5_shadow.py --stride 16 --exact 0 --probe 4000 --tag r03u_e0 > gpurun_out/r03u/c5_shadow_e0.log 2>&1 || { tail -5 gpurun_out/r03u/c5_shadow_e0.log; exit 1; }
tail -1 gpurun_out/r03u/c5_shadow_e0.log | cut -c1-700
