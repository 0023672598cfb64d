set -u
# every shadow query of the C5 frame vs brute force, exact-shadow mode and default
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r03q
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03q/pytest.log 2>&1 || { tail -40 gpurun_out/r03q/pytest.log; exit 1; }
tail -2 gpurun_out/r03q/pytest.log
for x in 1 0; do
  timeout -k 10 500 python -u tools/c5_shadow.py --stride 16 --all --exact $x --probe 4000 --tag r03q_e$x > gpurun_out/r03q/c5_shadow_e$x.log 2>&1 || { tail -5 gpurun_out/r03q/c5_shadow_e$x.log; exit 1; }
  tail -1 gpurun_out/r03q/c5_shadow_e$x.log | cut -c1-1500
done
