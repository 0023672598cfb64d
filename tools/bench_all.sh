#!/bin/bash
# Bench lines of every config: C1-C4 with the CPU
# baseline beside them, C2 also with the host octree.  Each run has its own
# time limit; the first failure ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-bench_all}
mkdir -p "$OUT"
run() {  # name, bench args...
  local name=$1; shift
  timeout -k 10 300 python3 bench.py "$@" > "$OUT/$name.json" 2> "$OUT/$name.err" || exit $?
  python3 -c "import json; d=json.load(open('$OUT/$name.json')); print('$name', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'])"
}
run c1 --workload c1 --steps 20 --warmup 2 --cpu-seconds 16
run c2_flat --workload c2 --steps 5 --warmup 1 --cpu-seconds 16
run c2_octree --workload c2 --accel octree --steps 10 --warmup 2 --cpu-seconds 16
run c3 --workload c3 --steps 20 --warmup 2 --cpu-seconds 16
run c4 --workload c4 --steps 20 --warmup 2 --cpu-seconds 16
