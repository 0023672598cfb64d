set -u
# device-length scans for the lists (RT_DEV_SCAN): parity subset, A/B against rocPRIM's scans, kernel trace
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r04r; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu.py -x -q --timeout 300 --timeout-method thread -k "cand or golden or exact or c5 or rank" > gpurun_out/r04r/pytest.log 2>&1 || { tail -40 gpurun_out/r04r/pytest.log; exit 1; }
tail -2 gpurun_out/r04r/pytest.log
VARIANTS="rocscan" WL=c5 bash tools/ab_bench.sh > gpurun_out/r04r/ab.log 2>&1 || { cat gpurun_out/r04r/ab.log; exit 1; }
cat gpurun_out/r04r/ab.log | cut -c1-160
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r04r/trace -o run --output-format csv -- python3 bench.py --no-cpu --steps 3 --warmup 1 > gpurun_out/r04r/trace.log 2>&1 || { tail -5 gpurun_out/r04r/trace.log; exit 1; }
python3 - <<'PY'
import csv, glob
f = glob.glob('gpurun_out/r04r/trace/**/*kernel_stats.csv', recursive=True)[0]
for r in csv.DictReader(open(f)):
    if 'scan' in r['Name'] or 'fillBuffer' in r['Name']:
        print(r['Name'][:60], r['Calls'], round(float(r['AverageNs'])/1e3, 1))
PY
timeout -k 10 300 python -u tools/rank_share.py --nranks 8 --steps 5 --out gpurun_out/r04r/rs8.json > gpurun_out/r04r/rs8.log 2>&1 || { tail -5 gpurun_out/r04r/rs8.log; exit 1; }
tail -2 gpurun_out/r04r/rs8.log | cut -c1-300
