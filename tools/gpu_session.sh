# one GPU session of round 6: config #5's write-back started from a hook on the rendered image's gradient (after the
# loss backward) against before loss.backward(); plain step times interleaved, then the kernel trace of each
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for m in 1 0 1 0 1 0; do
  HLGS_WB_HOOK=$m timeout -k 10 200 python3 tools/train_post_step.py --steps 30 > gpurun_out/wbh_$m.log 2>&1 || exit 1
  echo "hook=$m $(grep '^{' gpurun_out/wbh_$m.log | tail -1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["stages_ms"])')"
done
HLGS_WB_HOOK=1 bash tools/c5_trace.sh c5h1 | grep -i "ssim\|blend_bwd\|rows_packed\|preprocess\|ms_per_step" | cut -c1-200
HLGS_WB_HOOK=0 bash tools/c5_trace.sh c5h0 | grep -i "ssim\|blend_bwd\|rows_packed\|preprocess\|ms_per_step" | cut -c1-200
