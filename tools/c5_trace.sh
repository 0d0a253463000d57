# config #5 step under rocprofv3 --kernel-trace: per-kernel durations of the SPT-cache training step and, for the
# row-move kernels, how much of each launch overlapped another kernel (the write-back runs on a side stream).
#   bash tools/c5_trace.sh [tag]
set -eu
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${1:-c5}
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/$T -o run --output-format csv -- python3 tools/train_post_step.py --steps 20 > gpurun_out/$T.log 2>&1
python3 - gpurun_out/$T/run_kernel_trace.csv <<'PY'
import csv, sys, collections
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
iv = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows]
agg = collections.defaultdict(list)
for i, (s, e, n) in enumerate(iv):
    ov = 0
    for j in range(max(0, i - 50), min(len(iv), i + 50)):
        if j != i:
            s2, e2, _ = iv[j]
            ov += max(0, min(e, e2) - max(s, s2))
    agg[n.split("(")[0].replace("void ", "")].append(((e - s) / 1e3, min(ov, e - s) / 1e3))
tot = sorted(agg.items(), key=lambda kv: -sum(d for d, _ in kv[1]))
for n, v in tot[:25]:
    v = v[3:] if len(v) > 6 else v
    print(f"{sum(d for d, _ in v) / len(v):8.1f} us avg  overlapped {sum(o for _, o in v) / len(v):7.1f} us  n={len(v):3d}  {n[:90]}")
PY
grep "^{" gpurun_out/$T.log | tail -1 | cut -c1-600
