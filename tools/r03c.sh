set -u
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r03c
VARIANTS="sw4 sw8 tw5" bash tools/ab_bench.sh > gpurun_out/r03c/ab_occ.log 2>&1 || exit $?
for pol in 1 2 3; do
  timeout -k 10 200 python3 bench.py --no-cpu --steps 10 --warmup 2 --policy $pol > gpurun_out/r03c/pol$pol.json 2> gpurun_out/r03c/pol$pol.err || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/r03c/pol$pol.json')); r=d['roofline']; print('policy $pol', d['ms_per_step'], r['kernels_ms'])" >> gpurun_out/r03c/ab_occ.log
done
timeout -k 10 300 python3 tools/tile_cost.py --synthetic 32 --W 3840 --H 2160 --accel octree_gpu --out gpurun_out/r03c/tile_cost.json > gpurun_out/r03c/tile_cost.log 2>&1 || exit $?
cat gpurun_out/r03c/ab_occ.log
