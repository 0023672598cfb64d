set -u
# C1 / C3 kernel traces: where a small frame's time goes
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r04a; export TMPDIR=/tmp
for wl in c1 c3; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r04a/$wl -o run --output-format csv -- python3 bench.py --workload $wl --no-cpu --steps 20 --warmup 2 > gpurun_out/r04a/$wl.json 2> gpurun_out/r04a/$wl.err || { tail -5 gpurun_out/r04a/$wl.err; exit 1; }
  cut -c1-300 gpurun_out/r04a/$wl.json
done
