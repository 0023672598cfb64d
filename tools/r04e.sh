set -u
# packed candidate tests (RT_CAND_PK): parity subset, then A/B against the scalar loop
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r04e; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu.py -x -q --timeout 300 --timeout-method thread -k "cand or golden or exact or c5" > gpurun_out/r04e/pytest.log 2>&1 || { tail -40 gpurun_out/r04e/pytest.log; exit 1; }
tail -2 gpurun_out/r04e/pytest.log
VARIANTS="nopk" WL=c5 bash tools/ab_bench.sh > gpurun_out/r04e/ab.log 2>&1 || { cat gpurun_out/r04e/ab.log; exit 1; }
cat gpurun_out/r04e/ab.log | cut -c1-300
for v in default nopk; do python3 -c "import json; d=json.load(open('gpurun_out/ab/${v}_2.json')); r=d['roofline']; print('$v', {k: v['ms'] for k, v in r['kernels'].items()}, r['trace_phase_share'])"; done
