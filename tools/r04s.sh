set -u
# per-frame counters in one allocation / zeroed in quick_kernel: full GPU suite, smoke, A/B against the previous build
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r04s; export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04s/pytest.log 2>&1 || { tail -40 gpurun_out/r04s/pytest.log; exit 1; }
tail -2 gpurun_out/r04s/pytest.log
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r04s/smoke.log 2>&1 || { tail -20 gpurun_out/r04s/smoke.log; exit 1; }
tail -1 gpurun_out/r04s/smoke.log
VARIANTS="prev" WL=c5 bash tools/ab_bench.sh > gpurun_out/r04s/ab.log 2>&1 || { cat gpurun_out/r04s/ab.log; exit 1; }
VARIANTS="prev" WL=c5 bash tools/ab_bench.sh >> gpurun_out/r04s/ab.log 2>&1 || { cat gpurun_out/r04s/ab.log; exit 1; }
cat gpurun_out/r04s/ab.log | cut -c1-160
