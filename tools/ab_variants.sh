set -u
# A/B timing of libhlgs.so variants built by tools/build_variant.py (C = the in-tree build).  Each variant first
# passes the rasterizer parity tests, then the bench runs twice per variant, interleaved.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
V=hierarchical-lod-gaussians_amd/lib/variants
VARS="${VARIANTS:-A B C}"
for v in $VARS; do
  if [ $v = C ]; then L=""; else L=$V/$v.so; fi
  HLGS_LIBRARY=$L timeout -k 10 600 python -m pytest tests/test_gpu_parity.py tests/test_gpu_alt.py -q -x -p no:cacheprovider > gpurun_out/abt_$v.log 2>&1
  rc=$?; echo "$v tests rc=$rc $(tail -1 gpurun_out/abt_$v.log)"; [ $rc -eq 0 ] || exit $rc
done
for r in 1 2; do
for v in $VARS; do
  if [ $v = C ]; then L=""; else L=$V/$v.so; fi
  HLGS_LIBRARY=$L timeout -k 10 300 python bench.py --no-cpu-baseline --no-extras > gpurun_out/abc_$v$r.log 2>&1 || exit 1
  tail -1 gpurun_out/abc_$v$r.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); s=d['stages']; print('$v', d['value'], 'fwd', s['blend_fwd']['ms'], 'bwd', s['blend_bwd']['ms'], 'gauss', s['gauss_bwd']['ms'], 'pre', s['preprocess']['ms'])"
done; done
