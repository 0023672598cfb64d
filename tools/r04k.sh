set -u
# candidate tests without early exits (RT_CAND_NB): parity subset on the variant, A/B
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r04k; export TMPDIR=/tmp
RTGPU_LIB=raytracing-gpu_amd/lib/var_nb/librtgpu.so timeout -k 10 400 python -u -m pytest tests/test_gpu.py -x -q --timeout 300 --timeout-method thread -k "cand or golden or exact or c5" > gpurun_out/r04k/pytest.log 2>&1 || { tail -40 gpurun_out/r04k/pytest.log; exit 1; }
tail -2 gpurun_out/r04k/pytest.log
VARIANTS="nb" WL=c5 bash tools/ab_bench.sh > gpurun_out/r04k/ab.log 2>&1 || { cat gpurun_out/r04k/ab.log; exit 1; }
cat gpurun_out/r04k/ab.log | cut -c1-160
for v in default nb; do python3 -c "import json; d=json.load(open('gpurun_out/ab/${v}_2.json')); r=d['roofline']; print('$v', {k: v['ms'] for k, v in r['kernels'].items()}, r['trace_phase_share'])"; done
