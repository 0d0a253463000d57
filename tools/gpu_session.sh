# one GPU session of round 6: parity of the in-tree build (preprocess with one barrier: colour evaluated beside the
# geometry), then rocprof A/B against the two-barrier preprocess
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_alt.py tests/test_gpu_lod.py tests/test_gpu_dp.py tests/test_gpu_realcam.py -q -x -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/sess_tests.log 2>&1
rc=$?; echo "tests rc=$rc $(tail -1 gpurun_out/sess_tests.log)"; [ $rc -eq 0 ] || exit $rc
VARIANTS="C pre_2bar C pre_2bar" bash tools/ab_quick.sh
