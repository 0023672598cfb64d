set -u
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r03e
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03e/pytest.log 2>&1
rc=$?; tail -5 gpurun_out/r03e/pytest.log; echo "pytest rc=$rc"
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --no-cpu --steps 10 --warmup 2 > gpurun_out/r03e/bench_c5.json 2> gpurun_out/r03e/bench_c5.err || exit $?
cat gpurun_out/r03e/bench_c5.json
timeout -k 10 400 python -u tools/c5_shadow.py --stride 16 --tag r03e > gpurun_out/r03e/c5_shadow.log 2>&1 || exit $?
cat gpurun_out/r03e/c5_shadow.log
TAG=r03e_c5 bash tools/gpu_profile.sh > gpurun_out/r03e/profile.log 2>&1 || exit $?
tail -3 gpurun_out/r03e/profile.log
