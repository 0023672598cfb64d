set -u
# exact-shadow mode variants: band cosine split 1/n, 0.5/n; proof box 0.2x
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r03y
VARIANTS="band1 band05 box02" WL=c5 BENCH_EXTRA="--exact-shadows 1" bash tools/ab_bench.sh > gpurun_out/r03y/ab.log 2>&1 || { cat gpurun_out/r03y/ab.log; exit 1; }
cat gpurun_out/r03y/ab.log
for v in default band1 band05 box02; do python3 -c "import json; d=json.load(open('gpurun_out/ab/${v}_2.json')); r=d['roofline']; print('$v', {k: v['ms'] for k, v in r['kernels'].items()}, d['config']['accel_build']['light_buffer_entries'], r['per_lane']['shadow_tris_per_query'])"; done
