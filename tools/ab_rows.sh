# A/B of libhlgs.so variants (tools/build_variant.py; C = the in-tree build) on the SPT cache's row moves: the config5
# camera path under rocprofv3, per-call durations of k_rows_multi in step order (write-back, compaction, load).
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
V=hierarchical-lod-gaussians_amd/lib/variants
for v in ${VARIANTS:-C}; do
  if [ $v = C ]; then L=""; else L=$V/$v.so; fi
  HLGS_LIBRARY=$L timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/abr_$v -o run --output-format csv -- python3 tools/diag/cache_moves.py > gpurun_out/abr_$v.log 2>&1 || exit 1
  python3 - "$v" gpurun_out/abr_$v/run_kernel_trace.csv <<'PY'
import csv, sys
v, path = sys.argv[1:]
d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in csv.DictReader(open(path))
     if "k_rows_multi" in r["Kernel_Name"]]
legs = list(zip(*[d[i:i + 3] for i in range(3, len(d) - 2, 3)]))
print(v, " ".join(f"{name} {sum(x) / len(x):.1f}" for name, x in zip(("writeback", "compact", "load"), legs)))
PY
done
