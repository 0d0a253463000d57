# round 5 A/B: config #5 step with the in-tree library (C) and the 1024-thread binning variant (j1024), per-kernel
# averages under rocprofv3 for the binning kernels and the step time
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
V=hierarchical-lod-gaussians_amd/lib/variants
for v in C j1024 C j1024; do
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
