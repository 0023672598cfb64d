set -u
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r03m
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -x -v --timeout 200 --timeout-method thread -k "no_camera_lists or light_buffer or shadow_queries" > gpurun_out/r03m/pytest.log 2>&1 || { tail -40 gpurun_out/r03m/pytest.log; exit 1; }
tail -3 gpurun_out/r03m/pytest.log
timeout -k 10 1000 python -u tools/c5_exact.py --nranks 256 --ranks $RANKS --tag r03m_$PART > gpurun_out/r03m/c5_exact_$PART.log 2>&1
rc=$?; tail -2 gpurun_out/r03m/c5_exact_$PART.log | cut -c1-1500; exit $rc
