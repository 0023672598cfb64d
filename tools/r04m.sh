set -u
# final tree: GPU suite, smoke, default bench (CPU baseline), exact-shadow
# C5 bench, C1-C4 bench lines with their CPU baselines
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r04m; export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04m/pytest.log 2>&1 || { tail -40 gpurun_out/r04m/pytest.log; exit 1; }
tail -2 gpurun_out/r04m/pytest.log
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r04m/smoke.log 2>&1 || { tail -20 gpurun_out/r04m/smoke.log; exit 1; }
tail -1 gpurun_out/r04m/smoke.log
timeout -k 10 300 python3 bench.py > gpurun_out/r04m/bench_c5.json 2> gpurun_out/r04m/bench_c5.err || { tail -5 gpurun_out/r04m/bench_c5.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r04m/bench_c5.json')); print('c5', d['value'], d['ms_per_step'], d['roofline']['frac'], d['cpu_baseline']['value'])"
timeout -k 10 200 python3 bench.py --no-cpu --steps 10 --warmup 2 --exact-shadows 1 > gpurun_out/r04m/bench_c5_exact.json 2> gpurun_out/r04m/bench_c5_exact.err || { tail -5 gpurun_out/r04m/bench_c5_exact.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r04m/bench_c5_exact.json')); r=d['roofline']; print('exact', d['ms_per_step'], d['value'], {k: v['ms'] for k, v in r['kernels'].items()}, r['candidate_lists_ms'])"
for wl in c1 c2 c3 c4; do
  timeout -k 10 300 python3 bench.py --workload $wl --steps 10 --warmup 2 --cpu-seconds 12 > gpurun_out/r04m/bench_$wl.json 2> gpurun_out/r04m/bench_$wl.err || { tail -5 gpurun_out/r04m/bench_$wl.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r04m/bench_$wl.json')); r=d['roofline']; print('$wl', d['value'], d['ms_per_step'], {k: v['ms'] for k, v in r['kernels'].items()}, r.get('candidate_lists_ms'), (d.get('cpu_baseline') or {}).get('value'), (d.get('cpu_baseline') or {}).get('mode_a', {}).get('value'))"
done
