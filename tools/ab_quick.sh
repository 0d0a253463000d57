set -u
# Parity of the in-tree build (rasterizer + alt + configs tests), then rocprof kernel averages of each variant
# (tools/build_variant.py; C = the in-tree build):  VARIANTS="C old" bash tools/ab_quick.sh
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
V=hierarchical-lod-gaussians_amd/lib/variants
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_alt.py tests/test_gpu_configs.py -q -x -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/abq_tests.log 2>&1
rc=$?; echo "tests rc=$rc $(tail -1 gpurun_out/abq_tests.log)"; [ $rc -eq 0 ] || exit $rc
for v in ${VARIANTS:-C old}; do
  if [ $v = C ]; then L=""; else L=$V/$v.so; fi
  HLGS_LIBRARY=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/abq_$v -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-extras --no-stage-timing --steps 30 > gpurun_out/abq_$v.log 2>&1 || exit 1
  python3 - "$v" gpurun_out/abq_$v/run_kernel_stats.csv gpurun_out/abq_$v.log <<'PY'
import csv, json, sys
v, path, log = sys.argv[1:]
d = json.loads([l for l in open(log).read().splitlines() if l.startswith("{")][-1])
ks = {r["Name"].split("(")[0].replace("void ", ""): float(r["AverageNs"]) / 1e3 for r in csv.DictReader(open(path))}
print(v, d["value"], d["ms_per_step"], " ".join(f"{k.split('::')[-1]}={t:.1f}" for k, t in ks.items() if "hlgs" in k and t > 5))
PY
done
