# one GPU session of round 6: parity of the in-tree build (blend backward with the next batch's records prefetched,
# 4 waves per SIMD), then rocprof A/B against the 5-wave build (4 VGPRs spilled) and the previous kernel
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_plan.py tests/test_gpu_lod.py tests/test_gpu_alt.py -q -x -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/sess_tests.log 2>&1
rc=$?; echo "tests rc=$rc $(tail -1 gpurun_out/sess_tests.log)"; [ $rc -eq 0 ] || exit $rc
VARIANTS="C bwd_pf5 bwd_old C bwd_pf5 bwd_old" bash tools/ab_quick.sh
