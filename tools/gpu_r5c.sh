# round 5: full -m gpu suite on the in-tree build, then rocprof A/B (C = in-tree) of the variants in $VARIANTS
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_r5c.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_r5c.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
SKIP_TESTS=1 VARIANTS="${VARIANTS:-C}" bash tools/ab_prof.sh
