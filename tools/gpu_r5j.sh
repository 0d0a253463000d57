# round 5: which change moves test_configs4_merged_two_chunk_train_post_step[80k_leaves] -- the in-tree library, the
# round-4 SSIM kernels (oldloss), the binning without the wide-walk prefetch (prewide)
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
V=hierarchical-lod-gaussians_amd/lib/variants
T="tests/test_gpu_configs.py::test_configs4_merged_two_chunk_train_post_step"
for v in oldloss prewide C; do
  if [ $v = C ]; then L=""; else L=$V/$v.so; fi
  HLGS_LIBRARY=$L timeout -k 10 300 python -u -m pytest "$T" -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/r5j_$v.log 2>&1
  echo "$v rc=$?"; grep -E "^E .*ratio|passed|failed" gpurun_out/r5j_$v.log | head -3
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_loss.py tests/test_gpu_parity.py tests/test_gpu_alt.py -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r5j_rest.log 2>&1
echo "rest rc=$?"; tail -2 gpurun_out/r5j_rest.log
