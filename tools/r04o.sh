set -u
# radix bits per place of the lists' sort (RT_SORT_BITS 9: two places for 17-bit keys; 6): parity on s9, A/B
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r04o; export TMPDIR=/tmp
RTGPU_LIB=raytracing-gpu_amd/lib/var_s9/librtgpu.so timeout -k 10 400 python -u -m pytest tests/test_gpu.py -x -q --timeout 300 --timeout-method thread -k "cand or golden or c5 or rank" > gpurun_out/r04o/pytest.log 2>&1 || { tail -40 gpurun_out/r04o/pytest.log; exit 1; }
tail -2 gpurun_out/r04o/pytest.log
VARIANTS="s9 s6" WL=c5 bash tools/ab_bench.sh > gpurun_out/r04o/ab.log 2>&1 || { cat gpurun_out/r04o/ab.log; exit 1; }
cat gpurun_out/r04o/ab.log | cut -c1-160
RTGPU_LIB=raytracing-gpu_amd/lib/var_s9/librtgpu.so timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r04o/trace_s9 -o run --output-format csv -- python3 bench.py --no-cpu --steps 3 --warmup 1 > gpurun_out/r04o/trace_s9.log 2>&1 || { tail -5 gpurun_out/r04o/trace_s9.log; exit 1; }
python3 - <<'PY'
import csv, glob
f = glob.glob('gpurun_out/r04o/trace_s9/**/*kernel_stats.csv', recursive=True)[0]
for r in csv.DictReader(open(f)):
    if 'onesweep' in r['Name'] or 'radix' in r['Name']:
        print('s9', r['Name'][120:220], r['Calls'], round(float(r['AverageNs'])/1e3, 1))
PY
