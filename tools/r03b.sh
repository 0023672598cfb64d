set -u
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r03b
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03b/pytest.log 2>&1
rc=$?; tail -5 gpurun_out/r03b/pytest.log; echo "pytest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --no-cpu --steps 10 --warmup 2 > gpurun_out/r03b/bench_c5.json 2> gpurun_out/r03b/bench_c5.err
rc=$?; cat gpurun_out/r03b/bench_c5.json; tail -3 gpurun_out/r03b/bench_c5.err; echo "bench rc=$rc"
