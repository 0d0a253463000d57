# Round-end part A on the GPU box: the full -m gpu suite, smoke(), and config #5's kernel statistics
# (tools/gpu_c5prof.sh); part B is tools/profile_round.sh, the last GPU action of the round.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_all.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_all.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/smoke.log; exit 1; }
echo "smoke ok"
bash tools/gpu_c5prof.sh > gpurun_out/c5prof_summary.txt 2>&1
rc=$?; tail -3 gpurun_out/c5prof_summary.txt; exit $rc
