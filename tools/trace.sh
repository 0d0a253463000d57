set -eu
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/trace; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/trace -o run --output-format csv -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-extras --no-stage-timing > gpurun_out/trace/bench.log 2>&1
python3 tools/trace_gaps.py gpurun_out/trace/run_kernel_trace.csv
