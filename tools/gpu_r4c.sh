set -u
# Round 4: the full GPU suite on the in-tree build, then the timing A/B of the variants (tools/ab_prof.sh, no tests).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
  > gpurun_out/r4c_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc $(tail -1 gpurun_out/r4c_pytest.log)"; [ $rc -eq 0 ] || exit $rc
SKIP_TESTS=1 VARIANTS="${VARIANTS:-TL0 C}" bash tools/ab_prof.sh
