# round 5: SSIM in the round-4 summation order (horizontal in registers, vertical from LDS) -- the loss and config
# tests, then the whole GPU suite and the config #5 A/B
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_loss.py tests/test_gpu_configs.py -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_r5k.log 2>&1
rc=$?; echo "loss+configs rc=$rc"; tail -2 gpurun_out/pytest_r5k.log
[ $rc -eq 0 ] || { grep -E "^E |FAILED" gpurun_out/pytest_r5k.log | head -10; exit $rc; }
bash tools/gpu_r5g.sh && bash tools/gpu_r5i.sh
