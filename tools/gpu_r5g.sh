# round 5: SSIM two-pass kernels and the flat coarse cut -- loss, stream and cache GPU tests, then the config #5
# step under rocprofv3
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_loss.py tests/test_gpu_stream.py tests/test_gpu_cache.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_r5g.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_r5g.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" gpurun_out/pytest_r5g.log | head -20; exit $rc; }
bash tools/gpu_c5prof.sh
