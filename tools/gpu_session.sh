# one GPU session of round 6: the long-tile sort lengths test (tile lists across the block sort's size classes)
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "long_tile" -v -x -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/sess_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "PASS|FAIL|passed|failed|Error" gpurun_out/sess_tests.log | tail -8; exit $rc
