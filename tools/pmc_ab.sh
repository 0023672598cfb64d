#!/bin/bash
# SQ counters of the default build and each variant (lib/var_<name>), one
# PMC pass each (tools/pmc_pass.sh), the trace kernel's per-launch values.
#   VARIANTS="a b" gpurun -- bash tools/pmc_ab.sh <tag>
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; export TMPDIR=/tmp
T=${1:?tag}; O=gpurun_out/$T; mkdir -p $O
C=${CTRS:-"SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE"}
for v in default ${VARIANTS:-}; do
  if [ "$v" = default ]; then lib=""; else lib="raytracing-gpu_amd/lib/var_$v/librtgpu.so"; fi
  RTGPU_LIB=$lib bash tools/pmc_pass.sh $O/pmc_$v "$C" --workload ${WL:-c5} || { tail -20 $O/pmc_$v.log; exit 1; }
  python3 -c "import json; d=json.load(open('$O/pmc_$v.json')); k=d.get('${KERN:-trace_kernel}', {}); print('$v', json.dumps({c: round(x/1e6, 2) for c, x in k.items() if c != 'dispatches'}))"
done
