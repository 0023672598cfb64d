set -u
# depth-skip bounds read per prim in the trace kernel (RT_SKIP_BY_PRIM): parity on sp, A/B
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r04p; export TMPDIR=/tmp
RTGPU_LIB=raytracing-gpu_amd/lib/var_sp/librtgpu.so timeout -k 10 400 python -u -m pytest tests/test_gpu.py -x -q --timeout 300 --timeout-method thread -k "cand or golden or c5 or rank" > gpurun_out/r04p/pytest.log 2>&1 || { tail -40 gpurun_out/r04p/pytest.log; exit 1; }
tail -2 gpurun_out/r04p/pytest.log
VARIANTS="sp" WL=c5 bash tools/ab_bench.sh > gpurun_out/r04p/ab.log 2>&1 || { cat gpurun_out/r04p/ab.log; exit 1; }
cat gpurun_out/r04p/ab.log | cut -c1-160
RTGPU_LIB=raytracing-gpu_amd/lib/var_sp/librtgpu.so timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r04p/trace_sp -o run --output-format csv -- python3 bench.py --no-cpu --steps 3 --warmup 1 > gpurun_out/r04p/trace_sp.log 2>&1 || { tail -5 gpurun_out/r04p/trace_sp.log; exit 1; }
python3 - <<'PY'
import csv, glob
f = glob.glob('gpurun_out/r04p/trace_sp/**/*kernel_stats.csv', recursive=True)[0]
for r in csv.DictReader(open(f)):
    if 'trace_kernel' in r['Name'] or 'entry_skip' in r['Name']:
        print('sp', r['Name'][:60], r['Calls'], round(float(r['AverageNs'])/1e3, 1))
PY
