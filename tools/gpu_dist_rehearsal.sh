# Multi-rank bench rehearsal on a one-GPU box: two ranks share the card over gloo (the driver's N-GPU runs use RCCL,
# one rank per GPU); exercises bench.py's distributed path end to end (ring cameras, bucketed exchange, barriers,
# max-over-ranks timing, rank-0 line).
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
HLGS_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 5 --warmup 2 > gpurun_out/dist2.log 2>&1
rc=$?; echo "dist rc=$rc"; tail -4 gpurun_out/dist2.log; exit $rc
