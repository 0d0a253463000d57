# round 4: new parity tests at size, the plain bench (clock settle), the union-cut diagnostic
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_refparity.py tests/test_gpu_parity.py -v -x --timeout 600 --timeout-method thread -p no:cacheprovider > gpurun_out/r4a_tests.log 2>&1
rc=$?; grep -E "PASS|FAIL|ERROR|passed|failed" gpurun_out/r4a_tests.log | tail -40; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --no-cpu-baseline > gpurun_out/r4a_bench.log 2>&1 || exit 1
tail -1 gpurun_out/r4a_bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['launch_plan'], d['roofline']['kernel_ms'], {k: v['ms'] for k, v in d['stages'].items()})"
timeout -k 10 600 python -u tools/diag/union_cut.py --json gpurun_out/union_cut.json > gpurun_out/union_cut.log 2>&1 || { tail -20 gpurun_out/union_cut.log; exit 1; }
grep -v "^ \|^{\|^}" gpurun_out/union_cut.log | tail -10
