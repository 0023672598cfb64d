set -u
# small footprints counted and packed in one pass (small_pack): parity subset, A/B against the previous build
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r04u; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu.py -x -q --timeout 300 --timeout-method thread -k "cand or golden or exact or c5 or rank" > gpurun_out/r04u/pytest.log 2>&1 || { tail -40 gpurun_out/r04u/pytest.log; exit 1; }
tail -2 gpurun_out/r04u/pytest.log
VARIANTS="prev" WL=c5 bash tools/ab_bench.sh > gpurun_out/r04u/ab.log 2>&1 || { cat gpurun_out/r04u/ab.log; exit 1; }
VARIANTS="prev" WL=c5 bash tools/ab_bench.sh >> gpurun_out/r04u/ab.log 2>&1 || { cat gpurun_out/r04u/ab.log; exit 1; }
cat gpurun_out/r04u/ab.log | cut -c1-160
