# round 5: SSIM two-pass kernels, the flat coarse cut, the wide binning walk's prefetch -- the whole GPU suite, then
# the config #5 step under rocprofv3
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_r5g.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_r5g.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" gpurun_out/pytest_r5g.log | head -20; exit $rc; }
bash tools/gpu_c5prof.sh
