# LOD path loop: LOD GPU tests, then config #3 (tools/bench_extras.py --only lod) under rocprofv3 kernel stats.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_lod.py -q -x -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/lod_tests.log 2>&1
rc=$?; echo "lod tests rc=$rc"; tail -3 gpurun_out/lod_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/lodp -o run --output-format csv -- python3 tools/bench_extras.py --only lod > gpurun_out/lod_bench.log 2>&1 || exit 1
grep "^{" gpurun_out/lod_bench.log | tail -1
python3 - <<'PY'
import csv
for r in csv.DictReader(open("gpurun_out/lodp/run_kernel_stats.csv")):
    if "hlgs" in r["Name"]:
        print(f"{r['Name'].split('(')[0][:60]:60s} {r['Calls']:>5} {float(r['AverageNs'])/1e3:8.1f}us")
PY
