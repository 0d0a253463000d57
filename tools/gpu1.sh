set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests/test_gpu_parity.py -q -m gpu -p no:cacheprovider > gpurun_out/pytest1.log 2>&1
rc=$?
echo "pytest rc=$rc"
tail -30 gpurun_out/pytest1.log
if [ $rc -eq 0 ] || [ $rc -eq 1 ]; then
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-extras > gpurun_out/bench1.log 2>&1
  echo "bench rc=$?"
  tail -5 gpurun_out/bench1.log
fi
