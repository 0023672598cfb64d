set -u
# whole-frame C5 parity: octree_gpu (default: exact camera lists + light
# buffers) vs brute force over every tile of ranks RANKS of a 256-way split
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r03l
timeout -k 10 1080 python -u tools/c5_exact.py --nranks 256 --ranks $RANKS --tag r03l_$PART > gpurun_out/r03l/c5_exact_$PART.log 2>&1
rc=$?; tail -2 gpurun_out/r03l/c5_exact_$PART.log | cut -c1-1500; exit $rc
