# config #5 step under rocprofv3 --kernel-trace --stats: per-kernel averages of the SPT-cache training step
set -eu
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/c5prof -o run --output-format csv -- python3 tools/train_post_step.py --steps 20 > gpurun_out/c5prof.log 2>&1
python3 - gpurun_out/c5prof/run_kernel_stats.csv <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:30]:
    print(f'{float(r["TotalDurationNs"])/1e3/20:9.1f} us/step  {int(r["Calls"]):5d} calls  {float(r["AverageNs"])/1e3:8.1f} us  {r["Name"][:90]}')
PY
grep "^{" gpurun_out/c5prof.log | tail -1
