# one GPU session of round 6: the full -m gpu suite, then the default bench run (all legs)
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/sess_tests.log 2>&1
rc=$?; echo "tests rc=$rc $(tail -1 gpurun_out/sess_tests.log)"; [ $rc -eq 0 ] || { tail -30 gpurun_out/sess_tests.log; exit $rc; }
timeout -k 10 600 python bench.py > gpurun_out/bench_full.log 2>&1; rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || { tail -20 gpurun_out/bench_full.log; exit $rc; }
grep "^{" gpurun_out/bench_full.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read())
print(d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['frac'])
print('c3', d['config3']['inclusive_ms'], 'c4', d['config4_one_gpu']['ms_per_step'], 'c5', d['config5']['ms_per_step'], d['config5']['stages_ms'])
p=d['parity']; print('parity', p['color_linf'], p['pixels_above_1e-4'], p['grad_max_rel_err'], p['grad_elementwise_violations'])
print('cpu', d['cpu_baseline']['value'])
for k,v in d['stages'].items(): print(k, v)
"
