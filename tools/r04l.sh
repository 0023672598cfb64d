set -u
# light-buffer scans with the next record in flight (RT_LB_PREFETCH) at 8/6/5 waves: A/B
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r04l; export TMPDIR=/tmp
VARIANTS="pf8 pf6 pf5" WL=c5 bash tools/ab_bench.sh > gpurun_out/r04l/ab.log 2>&1 || { cat gpurun_out/r04l/ab.log; exit 1; }
cat gpurun_out/r04l/ab.log | cut -c1-160
for v in default pf8 pf6 pf5; do python3 -c "import json; d=json.load(open('gpurun_out/ab/${v}_2.json')); r=d['roofline']; print('$v', {k: v['ms'] for k, v in r['kernels'].items()})"; done
