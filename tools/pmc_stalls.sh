# Busy / stall / traffic PMC passes over a short bench run, one counter group per rocprofv3 pass (kernel-trace +
# --pmc only; never combined with sys/runtime traces).  Summarise with tools/summarize_stalls.py.
#   bash tools/pmc_stalls.sh <outdir> [extra bench args]
set -eu
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=${1:-gpurun_out/stall}
shift || true
mkdir -p $O
B=${PMC_CMD:-"python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-extras --no-stage-timing $*"}
run() { name=$1; shift
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc "$@" -d $O/$name -o run --output-format csv -- $B > $O/$name.log 2>&1
  echo "pass $name ok"; }
run p1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE GRBM_COUNT
run p2 SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INST_CYCLES_SALU
run p3 SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_MISC SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_ACTIVE_INST_FLAT
run fetch FETCH_SIZE
run write WRITE_SIZE
