# one GPU session of round 6: parity of the in-tree build, then rocprof A/B against the variants
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
VARIANTS="C pre_r6a C pre_r6a" bash tools/ab_quick.sh
