# one GPU session of round 6: the SPT cache tests, including the many-SPT cut (k_cache_lists' global search path)
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_cache.py -v -x -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/sess_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "PASS|FAIL|Error|passed|failed" gpurun_out/sess_tests.log | tail -15; exit $rc
