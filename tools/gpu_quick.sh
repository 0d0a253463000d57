# quick loop: gpu parity tests + bench (no cpu baseline), bench repeated to show run-to-run spread
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -q -m gpu -x -p no:cacheprovider > gpurun_out/pytest_q.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_q.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for i in 1 2 3; do
  timeout -k 10 400 python bench.py --no-cpu-baseline --no-extras "$@" > gpurun_out/bench_q$i.log 2>&1; rc=$?
  echo "bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
  tail -1 gpurun_out/bench_q$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], round(sum(v['ms'] for v in d['stages'].values()),4))"
done
tail -1 gpurun_out/bench_q3.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); [print(k, v) for k,v in d['stages'].items()]"
