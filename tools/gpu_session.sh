# one GPU session of round 6: bit-exact lists + parity of the in-tree build (split tile sort merged in registers),
# then rocprof A/B against the LDS merge-path build
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_plan.py tests/test_gpu_lod.py tests/test_gpu_scale.py tests/test_gpu_alt.py -q -x -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/sess_tests.log 2>&1
rc=$?; echo "tests rc=$rc $(tail -1 gpurun_out/sess_tests.log)"; [ $rc -eq 0 ] || exit $rc
VARIANTS="C sort_lds C sort_lds" bash tools/ab_quick.sh
