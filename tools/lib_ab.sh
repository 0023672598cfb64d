#!/bin/bash
# A/B of library builds: one bench line per build directory (RTGPU_LIB), an
# entry "dir:VAR=value" also setting one environment knob for that run.
# usage: LIBS="lib lib_v8 lib_v8:RT_SHADE_QUEUE=0" TAG=x ARGS="--steps 20 --warmup 3 --no-cpu" tools/lib_ab.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-libab}
mkdir -p $OUT
for ent in $LIBS; do
  l=${ent%%:*}; kv=""; [ "$ent" != "$l" ] && kv=${ent#*:}
  name=$(echo "$ent" | tr ':=' '__')
  env $kv RTGPU_LIB=raytracing-gpu_amd/$l/librtgpu.so timeout -k 10 ${BENCH_TIMEOUT:-240} python bench.py $ARGS > $OUT/$name.json 2> $OUT/$name.err
  rc=$?
  echo "$ent rc=$rc"
  python3 -c "import json;d=json.load(open('$OUT/$name.json'));r=d['roofline'];print(d['ms_per_step'], r['kernels']['trace']['ms'], r['kernels']['shade']['ms'], r['candidate_lists_ms'], 'fresh', d.get('ms_per_step_fresh'), (d.get('fresh_camera') or {}).get('candidate_lists_ms'))" || true
  if [ $rc -ne 0 ]; then exit $rc; fi
done
