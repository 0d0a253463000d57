# A/B of libhlgs.so variants on config #3 (tools/bench_extras.py --only lod) under rocprofv3 kernel stats; no tests
# (variants here may be deliberately wrong, e.g. cost floors).  C = the in-tree build.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
V=hierarchical-lod-gaussians_amd/lib/variants
for v in ${VARIANTS:-C}; do
  if [ $v = C ]; then L=""; else L=$V/$v.so; fi
  HLGS_LIBRARY=$L timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/ablod_$v -o run --output-format csv -- python3 tools/bench_extras.py --only lod > gpurun_out/ablod_$v.log 2>&1 || exit 1
  python3 - $v gpurun_out/ablod_$v/run_kernel_stats.csv <<'PY'
import csv, sys
ks = {r["Name"].split("(")[0].replace("void ", ""): float(r["AverageNs"]) / 1e3 for r in csv.DictReader(open(sys.argv[2]))}
print(sys.argv[1], " ".join(f"{k.split('::')[-1]}={t:.1f}" for k, t in ks.items() if "lerp" in k or "interp" in k))
PY
done
