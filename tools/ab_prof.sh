set -u
# A/B per-kernel durations of libhlgs.so variants (tools/build_variant.py; C = the in-tree build): parity tests
# first, then one rocprofv3 --kernel-trace --stats bench run per variant; prints the average per hlgs kernel.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
V=hierarchical-lod-gaussians_amd/lib/variants
VARS="${VARIANTS:-A B C}"
for v in $VARS; do
  [ "${SKIP_TESTS:-0}" = 1 ] && break  # timing-only diagnostic variants (parity deliberately broken)
  if [ $v = C ]; then L=""; else L=$V/$v.so; fi
  HLGS_LIBRARY=$L timeout -k 10 600 python -m pytest tests/test_gpu_parity.py tests/test_gpu_alt.py -q -x -p no:cacheprovider > gpurun_out/abt_$v.log 2>&1
  rc=$?; echo "$v tests rc=$rc $(tail -1 gpurun_out/abt_$v.log)"; [ $rc -eq 0 ] || exit $rc
done
for v in $VARS; do
  if [ $v = C ]; then L=""; else L=$V/$v.so; fi
  HLGS_LIBRARY=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/abp_$v -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-extras --no-stage-timing --steps 30 > gpurun_out/abp_$v.log 2>&1 || exit 1
  python3 - "$v" gpurun_out/abp_$v/run_kernel_stats.csv gpurun_out/abp_$v.log <<'PY'
import csv, json, sys
v, path, log = sys.argv[1:]
d = json.loads([l for l in open(log).read().splitlines() if l.startswith("{")][-1])
ks = {r["Name"].split("(")[0].replace("void ", ""): float(r["AverageNs"]) / 1e3 for r in csv.DictReader(open(path))}
print(v, d["value"], " ".join(f"{k.split('::')[-1]}={t:.1f}" for k, t in ks.items() if "hlgs" in k))
PY
done
