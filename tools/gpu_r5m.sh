# round 5 A/B: the headline bench with the in-tree library (C, 4,096 Gaussians per binning block at 1M) and with
# every binning block 2,048 Gaussians over 1024 threads (bg2048); parity tests first, then per-kernel averages
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
V=hierarchical-lod-gaussians_amd/lib/variants
HLGS_LIBRARY=$V/bg2048.so timeout -k 10 600 python -m pytest tests/test_gpu_parity.py tests/test_gpu_alt.py tests/test_gpu_plan.py -q -x -p no:cacheprovider > gpurun_out/abt_bg2048.log 2>&1
rc=$?; echo "bg2048 tests rc=$rc $(tail -1 gpurun_out/abt_bg2048.log)"; [ $rc -eq 0 ] || exit $rc
for v in C bg2048 C bg2048; do
  if [ $v = C ]; then L=""; else L=$V/$v.so; fi
  HLGS_LIBRARY=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/abh_$v -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extras --settle-max 30 > gpurun_out/abh_$v.log 2>&1 || exit 1
  python3 - "$v" gpurun_out/abh_$v/run_kernel_stats.csv gpurun_out/abh_$v.log <<'PY'
import csv, json, sys
v, path, log = sys.argv[1:]
rows = {r["Name"]: r for r in csv.DictReader(open(path))}
out = []
for key in ("k_count_tiles", "k_scatter_keys_lds", "k_tile_sort_wave", "k_tile_offsets_plan", "k_blend_fwd", "k_blend_bwd", "k_preprocess"):
    for n, r in rows.items():
        if key in n:
            out.append(f'{key}={float(r["AverageNs"]) / 1e3:.1f}')
line = [l for l in open(log) if l.startswith("{")][-1]
print(v, json.loads(line)["value"], " ".join(out))
PY
done
