set -u
# proven light buffers with origin bounds and band/cone choice: GPU suite,
# C5 A/B (slack vs proven), C5 shadow checks with adversarial probes
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r03o
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03o/pytest.log 2>&1 || { tail -40 gpurun_out/r03o/pytest.log; exit 1; }
tail -2 gpurun_out/r03o/pytest.log
for x in 0 1; do
  timeout -k 10 200 python3 bench.py --no-cpu --steps 10 --warmup 2 --exact-shadows $x > gpurun_out/r03o/bench_exact$x.json 2> gpurun_out/r03o/bench_exact$x.err || { tail -5 gpurun_out/r03o/bench_exact$x.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r03o/bench_exact$x.json')); r=d['roofline']; print('exact $x', d['ms_per_step'], {k: v['ms'] for k, v in r['kernels'].items()}, r['candidate_lists_ms'], d['config']['accel_build'], r['per_lane'])"
done
timeout -k 10 300 python -u tools/c5_shadow.py --stride 16 --exact 1 --probe 4000 --tag r03o_e1 > gpurun_out/r03o/c5_shadow_e1.log 2>&1 || { tail -5 gpurun_out/r03o/c5_shadow_e1.log; exit 1; }
cut -c1-2000 gpurun_out/r03o/c5_shadow_e1.log
for wl in c1 c2 c3 c4; do
  timeout -k 10 300 python3 bench.py --workload $wl --steps 10 --warmup 2 --cpu-seconds 12 > gpurun_out/r03o/bench_$wl.json 2> gpurun_out/r03o/bench_$wl.err || { tail -5 gpurun_out/r03o/bench_$wl.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r03o/bench_$wl.json')); print('$wl', d['value'], d['ms_per_step'], d['config'].get('accel'), (d.get('cpu_baseline') or {}).get('value'))"
done
