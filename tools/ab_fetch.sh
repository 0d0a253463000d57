# Traffic attribution of one kernel over libhlgs.so variants (tools/build_variant.py; C = in-tree): a FETCH_SIZE pass
# and a WRITE_SIZE pass per variant (separate --pmc runs, as MI355X_MICROARCH.md prescribes), per-launch bytes of the
# kernels matching KFILT (default k_blend_bwd): fetch = 2 x FETCH_SIZE (KiB -> bytes, gfx950 correction), write =
# WRITE_SIZE.   VARIANTS="C NG NP NS NW" bash tools/ab_fetch.sh
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
V=hierarchical-lod-gaussians_amd/lib/variants
B="python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-extras --no-stage-timing"
for v in ${VARIANTS:-C}; do
  if [ $v = C ]; then L=""; else L=$V/$v.so; fi
  for c in FETCH_SIZE WRITE_SIZE; do
    HLGS_LIBRARY=$L timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $c -d gpurun_out/abf_${v}_$c -o run --output-format csv -- $B > gpurun_out/abf_${v}_$c.log 2>&1 || exit 1
  done
  python3 - $v gpurun_out/abf_${v}_FETCH_SIZE/run_counter_collection.csv gpurun_out/abf_${v}_WRITE_SIZE/run_counter_collection.csv "${KFILT:-k_blend_bwd}" <<'PY'
import csv, sys, collections
v, pf, pw, kf = sys.argv[1:]
out = {}
for path, name, mul in ((pf, "fetch", 2 * 1024), (pw, "write", 1024)):
    acc = collections.defaultdict(float); n = collections.defaultdict(set)
    for r in csv.DictReader(open(path)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "")
        if kf not in k: continue
        acc[k] += float(r["Counter_Value"]); n[k].add(r["Dispatch_Id"])
    for k in acc:
        out.setdefault(k, {})[name] = acc[k] / len(n[k]) * mul / 1e6
for k, d in out.items():
    print(v, k, " ".join(f"{a}={b:.1f}MB" for a, b in d.items()))
PY
done
