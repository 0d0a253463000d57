# Round profile: FETCH_SIZE, WRITE_SIZE and SQ instruction counters in their own passes (never combined with
# sys/runtime traces), summarised on the box into profiles/r01/pmc_traffic.json so that the bench lines below
# report this build's traffic and instruction counts; then the bench under rocprofv3 kernel-trace/stats (the
# committed kernel statistics and the bench line of that same command), then a plain bench run.  Outputs land in
# gpurun_out/round/; copy them with tools/summarize_profile.py into profiles/<round>/.
set -eu
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/round
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $O/fetch -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-stage-timing > $O/fetch.log 2>&1
echo "fetch ok"
timeout -k 10 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $O/write -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-stage-timing > $O/write.log 2>&1
echo "write ok"
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES -d $O/sq -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-stage-timing > $O/sq.log 2>&1
echo "sq ok"
python3 tools/summarize_profile.py $O $O/summary > /dev/null
cp $O/summary/pmc_traffic.json profiles/r01/pmc_traffic.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 > $O/bench_line.log 2>&1
echo "trace ok"
timeout -k 10 300 python3 bench.py > $O/bench_plain.log 2>&1
echo "plain ok"
grep "^{" $O/bench_plain.log | tail -1
