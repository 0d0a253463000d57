# Round profile: FETCH_SIZE, WRITE_SIZE and SQ instruction counters in their own passes (never combined with
# sys/runtime traces), summarised on the box into profiles/<round>/pmc_traffic.json so that the bench lines below
# report this build's traffic and instruction counts; the busy / stall passes (tools/pmc_stalls.sh) summarised into
# profiles/<round>/stalls.json; then the bench step under rocprofv3 kernel-trace/stats (the committed kernel
# statistics and the bench line of that same command: --no-extras, so every launch of a kernel is the configs[1]
# frame), then the plain default bench run (all legs).  Outputs land in gpurun_out/round_<round>/, summaries in
# gpurun_out/round_<round>/summary/ (copy them into profiles/<round>/).
#   bash tools/profile_round.sh r02
set -eu
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R=${1:-r02}
O=gpurun_out/round_$R
mkdir -p $O profiles/$R
B="python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-extras --no-stage-timing"
timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $O/fetch -o run --output-format csv -- $B > $O/fetch.log 2>&1
echo "fetch ok"
timeout -k 10 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $O/write -o run --output-format csv -- $B > $O/write.log 2>&1
echo "write ok"
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES -d $O/sq -o run --output-format csv -- $B > $O/sq.log 2>&1
echo "sq ok"
python3 tools/summarize_profile.py $O $O/summary > /dev/null
cp $O/summary/pmc_traffic.json profiles/$R/pmc_traffic.json
bash tools/pmc_stalls.sh $O/stall
python3 tools/summarize_stalls.py $O/stall $O/summary/stalls.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-extras > $O/bench_line.log 2>&1
echo "trace ok"
timeout -k 10 400 python3 bench.py > $O/bench_plain.log 2>&1
echo "plain ok"
python3 tools/summarize_profile.py $O $O/summary > /dev/null
# only gpurun_out/ comes back from the box: copy $O/summary/* into profiles/$R/ afterwards
grep "^{" $O/bench_plain.log | tail -1
