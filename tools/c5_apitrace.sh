# config #5 step with the HIP runtime API traced beside the kernels: which host calls the GPU's idle gaps wait on.
#   bash tools/c5_apitrace.sh [tag]
set -eu
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${1:-c5api}
timeout -k 10 300 rocprofv3 --kernel-trace --hip-runtime-trace -d gpurun_out/$T -o run --output-format csv -- python3 tools/train_post_step.py --steps 8 > gpurun_out/$T.log 2>&1
ls gpurun_out/$T
