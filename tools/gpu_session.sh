# one GPU session of round 6: config #5 write-back placement x block count
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
V=hierarchical-lod-gaussians_amd/lib/variants
for cfg in "wb16 fwd" "wb24 fwd" "wb24 bwd" "wb16 start" "C start"; do
  set -- $cfg; v=$1; at=$2
  if [ $v = C ]; then L=""; else L=$V/$v.so; fi
  HLGS_LIBRARY=$L HLGS_WB_AT=$at timeout -k 10 300 python3 tools/train_post_step.py --steps 20 > gpurun_out/c5p_${v}_$at.log 2>&1 || exit 1
  echo "$v $at $(grep '^{' gpurun_out/c5p_${v}_$at.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['stages_ms'])")"
done
