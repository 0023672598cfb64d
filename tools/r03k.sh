set -u
# round 3, session 2: GPU suite, then the C5 profile (kernel trace, FETCH/WRITE,
# two SQ passes) and the bench line with the CPU baseline
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r03k
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r03k/pytest.log 2>&1 || { tail -40 gpurun_out/r03k/pytest.log; exit 1; }
tail -2 gpurun_out/r03k/pytest.log
TAG=r03k_c5 bash tools/gpu_profile.sh > gpurun_out/r03k/profile.log 2>&1 || { tail -30 gpurun_out/r03k/profile.log; exit 1; }
tail -3 gpurun_out/r03k/profile.log | cut -c1-3000
