# Round-end rehearsal on the GPU box: the full -m gpu suite, smoke(), then the profile round (PMC passes, stall
# passes, bench under rocprofv3 kernel-trace/stats, plain bench).
#   bash tools/round_check.sh r02
set -u
cd "$GRAFT_REPO_ROOT"
R=${1:-r02}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_all.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_all.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/smoke.log; exit 1; }
echo "smoke ok"
bash tools/profile_round.sh $R
