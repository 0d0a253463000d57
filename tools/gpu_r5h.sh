# round 5: busy / stall counters of the config #5 step (SPT cache + alt rasterizer), per kernel
set -eu
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
PMC_CMD="python3 tools/train_post_step.py --steps 4" bash tools/pmc_stalls.sh gpurun_out/c5stall
python3 tools/summarize_stalls.py gpurun_out/c5stall gpurun_out/c5stall.json > gpurun_out/c5stall_summary.txt 2>&1
python3 - <<'PY'
import json
d = json.load(open("gpurun_out/c5stall.json"))["kernels"]
for k, v in sorted(d.items(), key=lambda kv: -kv[1].get("pmc_pass_us", 0))[:14]:
    s = v.get("share_of_wave_time", {})
    print(f'{v.get("pmc_pass_us", 0):8.1f} us  waves/simd {v.get("waves_per_simd", 0):5.2f}  valu {v.get("valu_issue_frac", 0):4.2f}  '
          f'issue {s.get("issuing_any", 0):4.2f} wait {s.get("parked_waitcnt_barrier", 0):4.2f} stall {s.get("issue_stalled", 0):4.2f}  {k[:70]}')
PY
