set -u
cd "$GRAFT_REPO_ROOT"
R="$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof
timeout -k 10 900 python -m pytest tests -q -m gpu -p no:cacheprovider > gpurun_out/pytest2.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -25 gpurun_out/pytest2.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/smoke2.log 2>&1; echo "smoke rc=$?"; tail -3 gpurun_out/smoke2.log
timeout -k 10 400 python bench.py > gpurun_out/bench2.log 2>&1; rc=$?; echo "bench rc=$rc"; tail -2 gpurun_out/bench2.log
if [ $rc -ne 0 ]; then exit $rc; fi
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof" -o r1 -- python3 "$R/bench.py" --steps 10 --warmup 3 --no-cpu-baseline --no-extras > "$R/gpurun_out/prof_bench.log" 2>&1
echo "rocprof rc=$?"
find "$R/gpurun_out/prof" -name "*stats*" | head
