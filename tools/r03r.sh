set -u
# whole-frame C5 parity (default path): octree_gpu vs brute force over every
# tile of ranks RANKS of a 256-way split
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r03r
timeout -k 10 1050 python -u tools/c5_exact.py --nranks 256 --ranks $RANKS --tag r03r_$PART > gpurun_out/r03r/c5_exact_$PART.log 2>&1
rc=$?; tail -1 gpurun_out/r03r/c5_exact_$PART.log | cut -c1-600; exit $rc
