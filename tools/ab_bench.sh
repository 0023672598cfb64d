#!/bin/bash
# A/B of library variants on one workload: bench.py render-kernel time and
# frame time for the default build and each variant (lib/var_<name>), twice
# each, interleaved.  VARIANTS="name ..." WL=c5 bash tools/ab_bench.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab
WL=${WL:-c5}
for rep in 1 2; do
  for v in default ${VARIANTS:-}; do
    if [ "$v" = default ]; then lib=""; else lib="raytracing-gpu_amd/lib/var_$v/librtgpu.so"; fi
    RTGPU_LIB=$lib timeout -k 10 200 python3 bench.py --no-cpu --steps 10 --warmup 2 --workload $WL \
        ${BENCH_EXTRA:-} > gpurun_out/ab/${v}_$rep.json 2> gpurun_out/ab/${v}_$rep.err || exit $?
    python3 -c "import json; d=json.load(open('gpurun_out/ab/${v}_$rep.json')); r=d['roofline']; print('$v', $rep, 'frame_ms', d['ms_per_step'], 'kernel_ms', r['kernel_ms'], 'trace', r['kernels']['trace']['ms'], 'shade', r['kernels']['shade']['ms'], 'lists_ms', r['candidate_lists_ms'], 'Mrays', d['value'], 'grid', d['config']['accel_build'].get('persistent_grid'))"
  done
done
