# one GPU session of round 6: cache / stream tests of the in-tree build (pipelined k_cache_lists), then config #5
# kernel statistics of the in-tree build and of the previous k_cache_lists, interleaved
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_cache.py tests/test_gpu_stream.py tests/test_gpu_configs.py -q -x -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/sess_tests.log 2>&1
rc=$?; echo "tests rc=$rc $(tail -1 gpurun_out/sess_tests.log)"; [ $rc -eq 0 ] || exit $rc
V=hierarchical-lod-gaussians_amd/lib/variants
for v in C lists_old C lists_old; do
  if [ $v = C ]; then L=""; else L=$V/$v.so; fi
  HLGS_LIBRARY=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/c5l_$v -o run --output-format csv -- python3 tools/train_post_step.py --steps 20 > gpurun_out/c5l_$v.log 2>&1 || exit 1
  python3 - $v gpurun_out/c5l_$v/run_kernel_stats.csv gpurun_out/c5l_$v.log <<'PY'
import csv, json, sys
v, path, log = sys.argv[1:]
d = json.loads([l for l in open(log).read().splitlines() if l.startswith("{")][-1])
ks = {r["Name"].split("(")[0].replace("void ", ""): float(r["AverageNs"]) / 1e3 for r in csv.DictReader(open(path))}
print(v, d["ms_per_step"], d.get("stages_ms"), " ".join(f"{k.split('::')[-1]}={t:.1f}" for k, t in ks.items() if "cache" in k or "cut_flat" in k))
PY
done
