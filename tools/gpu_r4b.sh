set -u
# Round 4: list-parity tests of the in-tree build and the drop-empty variant, then the timing A/B (tools/ab_prof.sh).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
V=hierarchical-lod-gaussians_amd/lib/variants
for v in C DE; do
  if [ $v = C ]; then L=""; else L=$V/$v.so; fi
  HLGS_LIBRARY=$L timeout -k 10 600 python -u -m pytest tests/test_gpu_lod.py tests/test_gpu_realcam.py -x -q -p no:cacheprovider \
    --timeout 300 --timeout-method thread > gpurun_out/r4b_tests_$v.log 2>&1
  rc=$?; echo "$v list tests rc=$rc $(tail -1 gpurun_out/r4b_tests_$v.log)"; [ $rc -eq 0 ] || exit $rc
done
VARIANTS="${VARIANTS:-B0 C DE}" bash tools/ab_prof.sh
