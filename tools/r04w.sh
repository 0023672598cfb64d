set -u
# big-footprint row intervals kept for big_item_kernel: parity subset, A/B against the previous build
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r04w; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu.py -x -q --timeout 300 --timeout-method thread -k "cand or golden or exact or c5 or rank" > gpurun_out/r04w/pytest.log 2>&1 || { tail -40 gpurun_out/r04w/pytest.log; exit 1; }
tail -2 gpurun_out/r04w/pytest.log
VARIANTS="prev" WL=c5 bash tools/ab_bench.sh > gpurun_out/r04w/ab.log 2>&1 || { cat gpurun_out/r04w/ab.log; exit 1; }
VARIANTS="prev" WL=c5 bash tools/ab_bench.sh >> gpurun_out/r04w/ab.log 2>&1 || { cat gpurun_out/r04w/ab.log; exit 1; }
cat gpurun_out/r04w/ab.log | cut -c1-160
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r04w/trace -o run --output-format csv -- python3 bench.py --no-cpu --steps 3 --warmup 1 > gpurun_out/r04w/trace.log 2>&1 || { tail -5 gpurun_out/r04w/trace.log; exit 1; }
python3 - <<'PY'
import csv, glob
f = glob.glob('gpurun_out/r04w/trace/**/*kernel_stats.csv', recursive=True)[0]
for r in csv.DictReader(open(f)):
    if 'big_' in r['Name'] or 'count_kernel' in r['Name']:
        print(r['Name'][:50], r['Calls'], round(float(r['AverageNs'])/1e3, 1))
PY
