# A/B of libhlgs.so variants (tools/build_variant.py; C = the in-tree build) on config #5's step
# (tools/train_post_step.py under rocprofv3 kernel-trace/stats): the step time and the per-kernel averages.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
V=hierarchical-lod-gaussians_amd/lib/variants
for v in ${VARIANTS:-C}; do
  if [ $v = C ]; then L=""; else L=$V/$v.so; fi
  HLGS_LIBRARY=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/abt5_$v -o run --output-format csv -- python3 tools/train_post_step.py --steps 10 > gpurun_out/abt5_$v.log 2>&1 || exit 1
  python3 - "$v" gpurun_out/abt5_$v/run_kernel_stats.csv gpurun_out/abt5_$v.log <<'PY'
import csv, json, sys
v, path, log = sys.argv[1:]
d = json.loads([l for l in open(log).read().splitlines() if l.startswith("{")][-1])
ks = sorted(csv.DictReader(open(path)), key=lambda r: -float(r["TotalDurationNs"]))
print(v, d["ms_per_step"], d["stages_ms"])
print("   ", " ".join(f'{r["Name"].split("(")[0].replace("void ", "").split("::")[-1]}={float(r["AverageNs"]) / 1e3:.1f}' for r in ks[:12]))
PY
done
