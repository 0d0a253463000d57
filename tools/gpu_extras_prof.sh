# Kernel statistics of the driver line's other legs on the final library: configs[2] (the LOD chain,
# tools/bench_extras.py --only lod) and configs[3]'s per-GPU frame (bench.py --P 4000000) under rocprofv3.
set -eu
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/x_lod -o run --output-format csv -- python3 tools/bench_extras.py --only lod > gpurun_out/x_lod.log 2>&1
echo "lod ok"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/x_c4 -o run --output-format csv -- python3 bench.py --P 4000000 --steps 10 --warmup 3 --no-extras --no-cpu-baseline --no-stage-timing > gpurun_out/x_c4.log 2>&1
echo "c4 ok"
grep "^{" gpurun_out/x_c4.log | tail -1 | cut -c1-300
