set -u
# r04c (full validation), then an A/B of the split kernels' occupancy targets
cd $GRAFT_REPO_ROOT
bash tools/r04c.sh || exit 1
VARIANTS="sw6 sw7 tw4" WL=c5 bash tools/ab_bench.sh > gpurun_out/r04c/ab.log 2>&1 || { cat gpurun_out/r04c/ab.log; exit 1; }
cat gpurun_out/r04c/ab.log | cut -c1-300
for v in default sw6 sw7 tw4; do python3 -c "import json; d=json.load(open('gpurun_out/ab/${v}_2.json')); r=d['roofline']; print('$v', {k: v['ms'] for k, v in r['kernels'].items()})"; done
