# A/B of libhlgs.so variants (tools/build_variant.py; C = the in-tree build) on the SPT cache's row moves: the config5
# camera path under rocprofv3, mean per-call durations of the legs (upper cut, write-back k_rows_packed<true>, compaction
# k_rows_compact or k_rows_multi, load k_rows_packed<false>) over the steps after the first.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
V=hierarchical-lod-gaussians_amd/lib/variants
for v in ${VARIANTS:-C}; do
  if [ $v = C ]; then L=""; else L=$V/$v.so; fi
  HLGS_LIBRARY=$L timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/abr_$v -o run --output-format csv -- python3 tools/diag/cache_moves.py > gpurun_out/abr_$v.log 2>&1 || exit 1
  python3 - "$v" gpurun_out/abr_$v/run_kernel_trace.csv <<'PY'
import csv, sys
v, path = sys.argv[1:]
rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
legs = {"upper_cut": [], "writeback": [], "compact": [], "load": []}
for r in rows:
    n, d = r["Kernel_Name"], (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    if "k_upper_cut" in n: legs["upper_cut"].append(d)
    elif "k_rows_packed<true>" in n: legs["writeback"].append(d)
    elif "k_rows_multi" in n or "k_rows_compact" in n: legs["compact"].append(d)
    elif "k_rows_packed<false>" in n: legs["load"].append(d)
skip = {"upper_cut": 1, "writeback": 0, "compact": 0, "load": 2}  # setup head load and the first step's full load
print(v, " ".join(f"{k} {sum(x[skip[k]:]) / max(1, len(x[skip[k]:])):.1f} (n={len(x)})" for k, x in legs.items()))
PY
done
