set -u
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r03d gpurun_out/r03c
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03d/pytest.log 2>&1
rc=$?; tail -5 gpurun_out/r03d/pytest.log; echo "pytest rc=$rc"
if [ $rc -ne 0 ]; then exit $rc; fi
bash tools/r03c.sh
