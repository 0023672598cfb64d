set -u
# shared reciprocals in the lists fast path: parity subset, then A/B against the IEEE-division build
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r04g; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu.py -x -q --timeout 300 --timeout-method thread -k "cand or golden or exact or c5 or rank" > gpurun_out/r04g/pytest.log 2>&1 || { tail -40 gpurun_out/r04g/pytest.log; exit 1; }
tail -2 gpurun_out/r04g/pytest.log
VARIANTS="divs" WL=c5 bash tools/ab_bench.sh > gpurun_out/r04g/ab.log 2>&1 || { cat gpurun_out/r04g/ab.log; exit 1; }
cat gpurun_out/r04g/ab.log | cut -c1-300
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r04g/trace -o run --output-format csv -- python3 bench.py --no-cpu --steps 5 --warmup 1 > gpurun_out/r04g/trace.log 2>&1 || { tail -5 gpurun_out/r04g/trace.log; exit 1; }
python3 - <<'PY'
import csv, glob
f = glob.glob('gpurun_out/r04g/trace/**/*kernel_stats.csv', recursive=True)[0]
for r in sorted(csv.DictReader(open(f)), key=lambda r: -float(r['TotalDurationNs']))[:16]:
    print(r['Name'][:60], r['Calls'], round(float(r['AverageNs'])/1e3, 1))
PY
