# round 5: 1024-thread binning blocks and the flat cut's separate write kernel -- the whole GPU suite, then the
# config #5 step under rocprofv3 (per-kernel averages)
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_r5l.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_r5l.log
[ $rc -eq 0 ] || { grep -E "^E |FAILED" gpurun_out/pytest_r5l.log | head -10; exit $rc; }
bash tools/gpu_c5prof.sh
