# round 5: the SPT-cache GPU tests, then the config #5 step under rocprofv3 (per-kernel averages)
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_cache.py tests/test_gpu_stream.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_r5e.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_r5e.log
[ $rc -eq 0 ] || exit $rc
bash tools/gpu_c5prof.sh
