# round 5 A/B: config #5 step with the in-tree library (C) and 1,024 Gaussians per binning block below 819,200 (bg1024), per-kernel
# averages under rocprofv3 for the binning kernels and the step time
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
V=hierarchical-lod-gaussians_amd/lib/variants
HLGS_LIBRARY=$V/bg1024.so timeout -k 10 600 python -m pytest tests/test_gpu_parity.py tests/test_gpu_alt.py tests/test_gpu_plan.py tests/test_gpu_cache.py -q -x -p no:cacheprovider > gpurun_out/abt_bg1024.log 2>&1
rc=$?; echo "bg1024 tests rc=$rc $(tail -1 gpurun_out/abt_bg1024.log)"; [ $rc -eq 0 ] || exit $rc
for v in C bg1024 C bg1024; do
  if [ $v = C ]; then L=""; else L=$V/$v.so; fi
  HLGS_LIBRARY=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/ab_$v -o run --output-format csv -- python3 tools/train_post_step.py --steps 20 > gpurun_out/ab_$v.log 2>&1 || exit 1
  python3 - "$v" gpurun_out/ab_$v/run_kernel_stats.csv gpurun_out/ab_$v.log <<'PY'
import csv, json, sys
v, path, log = sys.argv[1:]
rows = {r["Name"]: r for r in csv.DictReader(open(path))}
out = []
for key in ("k_count_tiles", "k_scatter_keys_lds", "k_tile_sort_wave", "k_tile_offsets_plan", "k_blend_fwd", "k_ssim_fwd", "k_ssim_bwd", "k_cut_flat", "k_upper_cut", "k_cut_level"):
    for n, r in rows.items():
        if key in n:
            out.append(f'{key}={float(r["AverageNs"]) / 1e3:.1f}')
line = [l for l in open(log) if l.startswith("{")][-1]
print(v, json.loads(line)["ms_per_step"], " ".join(out))
PY
done
