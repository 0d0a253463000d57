# one GPU session of round 6: cache tests, then the config #5 trace with the deferred write-back
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_cache.py tests/test_gpu_stream.py tests/test_gpu_act.py tests/test_gpu_loss.py tests/test_gpu_configs.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/sess_tests.log 2>&1
rc=$?; echo "tests rc=$rc $(tail -1 gpurun_out/sess_tests.log)"; [ $rc -eq 0 ] || { tail -30 gpurun_out/sess_tests.log; exit $rc; }
bash tools/c5_trace.sh c5d | cut -c1-220
