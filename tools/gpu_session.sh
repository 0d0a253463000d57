# one GPU session of round 6: rocprof A/B of the in-tree build against cost-floor variants
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
VARIANTS="C sort_nonet sort_nomerge" bash tools/ab_quick.sh
