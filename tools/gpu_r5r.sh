# round 5 final: the default bench line (all legs) and smoke
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r5r.txt 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/smoke_r5r.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python3 bench.py > gpurun_out/bench_r5r.log 2>&1
rc=$?; echo "bench rc=$rc"; grep "^{" gpurun_out/bench_r5r.log | tail -1 | cut -c1-300
