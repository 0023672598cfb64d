set -u
# full validation of the committed tree: GPU suite, smoke, default bench (with
# the CPU baseline), and the all-query shadow check in both shadow modes
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r04c; export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04c/pytest.log 2>&1 || { tail -40 gpurun_out/r04c/pytest.log; exit 1; }
tail -2 gpurun_out/r04c/pytest.log
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r04c/smoke.log 2>&1 || { tail -20 gpurun_out/r04c/smoke.log; exit 1; }
tail -1 gpurun_out/r04c/smoke.log
timeout -k 10 300 python3 bench.py > gpurun_out/r04c/bench.json 2> gpurun_out/r04c/bench.err || { tail -5 gpurun_out/r04c/bench.err; exit 1; }
cut -c1-600 gpurun_out/r04c/bench.json
for x in 0 1; do
  timeout -k 10 300 python -u tools/c5_shadow.py --stride 16 --exact $x --probe 4000 --tag r04c_e$x > gpurun_out/r04c/c5_shadow_e$x.log 2>&1 || { tail -5 gpurun_out/r04c/c5_shadow_e$x.log; exit 1; }
  tail -1 gpurun_out/r04c/c5_shadow_e$x.log | cut -c1-500
done
