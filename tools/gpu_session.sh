# one GPU session of round 6: the config #5 trace with the write-back flushed before the backward
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
bash tools/c5_trace.sh c5e | cut -c1-220
