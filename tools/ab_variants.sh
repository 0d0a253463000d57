set -u
# A/B timing of libhlgs.so variants built by tools/build_variant.py (C = the in-tree build)
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
V=hierarchical-lod-gaussians_amd/lib/variants
for r in 1 2; do
for v in A B C; do
  if [ $v = C ]; then L=""; else L=$V/$v.so; fi
  HLGS_LIBRARY=$L timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/abc_$v$r.log 2>&1 || exit 1
  tail -1 gpurun_out/abc_$v$r.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', d['value'], d['stages']['blend_bwd']['ms'], d['roofline']['kernel_ms'])"
done; done
