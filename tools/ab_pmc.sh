# A/B of SQ instruction / activity counters for libhlgs.so variants (tools/build_variant.py; C = in-tree build):
# one --pmc pass per variant over a short bench run, per-launch averages of the kernels matching KFILT (blend).
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
V=hierarchical-lod-gaussians_amd/lib/variants
B="python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-extras --no-stage-timing"
for v in ${VARIANTS:-C}; do
  if [ $v = C ]; then L=""; else L=$V/$v.so; fi
  HLGS_LIBRARY=$L timeout -k 10 300 rocprofv3 --kernel-trace --pmc ${PMC:-SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU} \
    -d gpurun_out/abpmc_$v -o run --output-format csv -- $B > gpurun_out/abpmc_$v.log 2>&1 || exit 1
  python3 - $v gpurun_out/abpmc_$v/run_counter_collection.csv "${KFILT:-blend}" <<'PY'
import csv, sys, collections
v, path, kf = sys.argv[1:]
acc = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.defaultdict(set)
for r in csv.DictReader(open(path)):
    k = r["Kernel_Name"].split("(")[0].replace("void ", "").split("::")[-1]
    if kf not in k: continue
    acc[k][r["Counter_Name"]] += float(r["Counter_Value"]); n[k].add(r["Dispatch_Id"])
for k, c in acc.items():
    print(v, k, " ".join(f"{name}={val / len(n[k]):.4g}" for name, val in sorted(c.items())))
PY
done
