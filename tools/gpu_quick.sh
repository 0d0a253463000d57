# quick loop: gpu parity tests + bench (no cpu baseline)
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -q -m gpu -x -p no:cacheprovider > gpurun_out/pytest_q.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_q.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python bench.py --no-cpu-baseline "$@" > gpurun_out/bench_q.log 2>&1; rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench_q.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step']); [print(k, v) for k,v in d['stages'].items()]"
