# exactness + cost runs on the GPU box (one call): tools/c5_exact.py and
# rocprofv3 kernel traces of tools/prof_render.py
export TMPDIR=/tmp; mkdir -p gpurun_out
R=$(pwd)
run() { tag=$1; shift; timeout -k 10 500 python -u tools/c5_exact.py --tag $tag "$@" > gpurun_out/$tag.log 2>&1; }
prof() { tag=$1; shift; (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_$tag -o run --output-format csv -- python3 $R/tools/prof_render.py "$@" > $R/gpurun_out/prof_$tag.log 2>&1); }
eval "${RUNS:-true}"
rc=$?; for f in gpurun_out/*.log; do echo == $f; grep -v '^{' $f | grep -v "^W2026\|^I2026\|^E2026" | tail -4; done; exit $rc
