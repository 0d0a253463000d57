# round 5: wide record sums two Gaussians per pass -- the whole GPU suite, then config #5 A/B against the
# previous commit's library (head) under rocprofv3
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_alt.py tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_cache.py -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_r5w.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_r5w.log
[ $rc -eq 0 ] || { grep -E "^E |FAILED" gpurun_out/pytest_r5w.log | head -10; exit $rc; }
V=hierarchical-lod-gaussians_amd/lib/variants
for v in head C head C; do
  if [ $v = C ]; then L=""; else L=$V/$v.so; fi
  HLGS_LIBRARY=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/ab_$v -o run --output-format csv -- python3 tools/train_post_step.py --steps 20 > gpurun_out/ab_$v.log 2>&1 || exit 1
  python3 - "$v" gpurun_out/ab_$v/run_kernel_stats.csv gpurun_out/ab_$v.log <<'PY'
import csv, json, sys
v, path, log = sys.argv[1:]
rows = {r["Name"]: r for r in csv.DictReader(open(path))}
out = []
for key in ("k_gauss_bwd", "k_count_tiles", "k_scatter_keys_lds"):
    for n, r in rows.items():
        if key in n:
            out.append(f'{key}={float(r["AverageNs"]) / 1e3:.1f}')
line = [l for l in open(log) if l.startswith("{")][-1]
print(v, json.loads(line)["ms_per_step"], " ".join(out))
PY
done
