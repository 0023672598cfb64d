set -u
# inline candidate records: GPU suite, C5 bench x2
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r03z
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03z/pytest.log 2>&1 || { tail -40 gpurun_out/r03z/pytest.log; exit 1; }
tail -2 gpurun_out/r03z/pytest.log
for i in 1 2; do
  timeout -k 10 200 python3 bench.py --no-cpu --steps 10 --warmup 2 > gpurun_out/r03z/bench_$i.json 2> gpurun_out/r03z/bench_$i.err || { tail -5 gpurun_out/r03z/bench_$i.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r03z/bench_$i.json')); r=d['roofline']; print('c5', d['ms_per_step'], d['value'], {k: v['ms'] for k, v in r['kernels'].items()}, r['candidate_lists_ms'])"
done
