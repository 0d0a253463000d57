# One build -> measure iteration on the GPU box: GPU tests (optionally a subset), a plain bench line, and the bench
# under rocprofv3 kernel-trace/stats; prints the bench line and the hlgs kernel averages.
#   bash tools/gpu_iter.sh <tag> [pytest selection...]
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
T=${1:-iter}; shift || true
O=gpurun_out/$T
mkdir -p $O
SEL="${*:-tests}"
timeout -k 10 600 python -u -m pytest $SEL -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -4 $O/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline --no-extras > $O/bench.log 2>&1 || { echo "bench failed"; tail -20 $O/bench.log; exit 1; }
grep "^{" $O/bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('value', d['value'], 'ms', d['ms_per_step']); [print(' ', k, v) for k,v in d['stages'].items()]"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-extras --no-stage-timing --steps 30 > $O/prof.log 2>&1 || { echo "rocprof failed"; exit 1; }
python3 - $O/prof/run_kernel_stats.csv <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "hlgs" in r["Name"]:
        print(f'{float(r["AverageNs"])/1e3:9.1f} us  x{r["Calls"]:>4}  {r["Name"].split("(")[0].replace("void ", "")}')
PY
