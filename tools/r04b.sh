set -u
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r04b; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu.py -x -q --timeout 300 --timeout-method thread -k "shadow or light_buffer or golden" > gpurun_out/r04b/pytest.log 2>&1 || { tail -40 gpurun_out/r04b/pytest.log; exit 1; }
tail -2 gpurun_out/r04b/pytest.log
VARIANTS="spf" WL=c5 bash tools/ab_bench.sh > gpurun_out/r04b/ab.log 2>&1 || { cat gpurun_out/r04b/ab.log; exit 1; }
cat gpurun_out/r04b/ab.log
for v in default spf; do python3 -c "import json; d=json.load(open('gpurun_out/ab/${v}_2.json')); r=d['roofline']; print('$v', {k: v['ms'] for k, v in r['kernels'].items()})"; done
bash tools/r04a.sh
