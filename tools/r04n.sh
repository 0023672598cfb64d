set -u
# workgroup size of the per-prim list passes (RT_LIST_BLOCK 64/128/256/512): A/B with kernel times
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r04n; export TMPDIR=/tmp
VARIANTS="b64 b128 b512" WL=c5 bash tools/ab_bench.sh > gpurun_out/r04n/ab.log 2>&1 || { cat gpurun_out/r04n/ab.log; exit 1; }
cat gpurun_out/r04n/ab.log | cut -c1-160
for v in b64 b512; do
  RTGPU_LIB=raytracing-gpu_amd/lib/var_$v/librtgpu.so timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r04n/trace_$v -o run --output-format csv -- python3 bench.py --no-cpu --steps 3 --warmup 1 > gpurun_out/r04n/trace_$v.log 2>&1 || { tail -5 gpurun_out/r04n/trace_$v.log; exit 1; }
done
python3 - <<'PY'
import csv, glob
for v in ('b64', 'b512'):
    f = glob.glob('gpurun_out/r04n/trace_%s/**/*kernel_stats.csv' % v, recursive=True)[0]
    for r in csv.DictReader(open(f)):
        if any(k in r['Name'] for k in ('quick_kernel', 'rtc::count_kernel', 'rtc::emit_kernel')):
            print(v, r['Name'][:40], r['Calls'], round(float(r['AverageNs'])/1e3, 1))
PY
