# one GPU session of round 6: parity of the in-tree build (long-tile block sort split into 2,048- and 4,096-key LDS instances), then
# rocprof A/B on config #4's per-GPU frame (4M Gaussians) against the LDS bitonic block sort
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_plan.py tests/test_gpu_scale.py tests/test_gpu_configs.py -q -x -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/sess_tests.log 2>&1
rc=$?; echo "tests rc=$rc $(tail -1 gpurun_out/sess_tests.log)"; [ $rc -eq 0 ] || exit $rc
V=hierarchical-lod-gaussians_amd/lib/variants
for v in C sort_m3 C sort_m3; do
  if [ $v = C ]; then L=""; else L=$V/$v.so; fi
  HLGS_LIBRARY=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/c4s_$v -o run --output-format csv -- python3 bench.py --P 4000000 --steps 10 --warmup 3 --no-extras --no-cpu-baseline --no-stage-timing > gpurun_out/c4s_$v.log 2>&1 || exit 1
  python3 - "$v" gpurun_out/c4s_$v/run_kernel_stats.csv gpurun_out/c4s_$v.log <<'PY'
import csv, json, sys
v, path, log = sys.argv[1:]
d = json.loads([l for l in open(log).read().splitlines() if l.startswith("{")][-1])
ks = {r["Name"].split("(")[0].replace("void ", ""): float(r["AverageNs"]) / 1e3 for r in csv.DictReader(open(path))}
print(v, d["value"], d["ms_per_step"], " ".join(f"{k.split('::')[-1]}={t:.1f}" for k, t in ks.items() if "sort" in k or "merge" in k or "blend" in k))
PY
done
