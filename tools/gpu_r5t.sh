# round 5 final check: the whole GPU suite on the final build
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_r5t.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_r5t.log
[ $rc -eq 0 ] || { grep -E "^E |FAILED" gpurun_out/pytest_r5t.log | head -10; exit $rc; }
