# Rehearsal of bench.py's view-data-parallel config #5 leg on a one-GPU box: two ranks share the card over gloo
# (the driver's N-GPU runs use RCCL, one rank per GPU); the config #4 exchange (944 MB over gloo) is skipped and config #5 runs at 200k leaves for 2 timed steps.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
HLGS_DIST_BACKEND=gloo HLGS_BENCH_SKIP_CONFIG4=1 HLGS_BENCH_CONFIG5_STEPS=2 HLGS_BENCH_CONFIG5_P=200000 HLGS_BENCH_TRACE=1 timeout -k 10 400 \
  python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 \
  bench.py --gpus 2 --steps 5 --warmup 2 > gpurun_out/dist2_c5.log 2>&1
rc=$?; echo "dist rc=$rc"; tail -3 gpurun_out/dist2_c5.log | cut -c1-400; exit $rc
