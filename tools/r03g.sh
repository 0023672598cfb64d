set -u
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r03g
timeout -k 10 300 python -u tools/c5_shadow.py --stride 16 --tag r03g > gpurun_out/r03g/c5_shadow.log 2>&1 || exit $?
cat gpurun_out/r03g/c5_shadow.log
timeout -k 10 1000 python -u tools/c5_exact.py --nranks 256 --ranks 0-255 --tag r03g > gpurun_out/r03g/c5_exact.log 2>&1
rc=$?; tail -3 gpurun_out/r03g/c5_exact.log | cut -c1-1500; exit $rc
