set -u
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r03f
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03f/pytest.log 2>&1
rc=$?; tail -5 gpurun_out/r03f/pytest.log; echo "pytest rc=$rc"
if [ $rc -ne 0 ]; then exit $rc; fi
VARIANTS="cand0 tw6" bash tools/ab_bench.sh > gpurun_out/r03f/ab.log 2>&1 || exit $?
cat gpurun_out/r03f/ab.log
for wl in c4 c3 c2 c1; do
  timeout -k 10 300 python -u bench.py --no-cpu --steps 10 --warmup 2 --workload $wl > gpurun_out/r03f/bench_$wl.json 2> gpurun_out/r03f/bench_$wl.err || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/r03f/bench_$wl.json')); r=d['roofline']; print('$wl', d['ms_per_step'], d['value'], r['kernels'])"
done
timeout -k 10 300 python -u tools/rank_share.py --nranks 1 2 4 8 --all-ranks --steps 5 --out gpurun_out/r03f/rank_share.json > gpurun_out/r03f/rank_share.log 2>&1 || exit $?
tail -20 gpurun_out/r03f/rank_share.log
timeout -k 10 300 python -u tools/noground.py --out gpurun_out/r03f/noground.json > gpurun_out/r03f/noground.log 2>&1 || exit $?
tail -2 gpurun_out/r03f/noground.log | cut -c1-400
TAG=r03f_c5 bash tools/gpu_profile.sh > gpurun_out/r03f/profile.log 2>&1 || exit $?
tail -3 gpurun_out/r03f/profile.log | cut -c1-300
