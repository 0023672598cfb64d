set -u
# final tree: GPU suite, smoke, default bench line (with its CPU baseline)
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r04v; export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04v/pytest.log 2>&1 || { tail -40 gpurun_out/r04v/pytest.log; exit 1; }
tail -2 gpurun_out/r04v/pytest.log
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r04v/smoke.log 2>&1 || { tail -20 gpurun_out/r04v/smoke.log; exit 1; }
tail -1 gpurun_out/r04v/smoke.log
timeout -k 10 300 python3 bench.py > gpurun_out/r04v/bench.json 2> gpurun_out/r04v/bench.err || { tail -5 gpurun_out/r04v/bench.err; exit 1; }
cut -c1-400 gpurun_out/r04v/bench.json
