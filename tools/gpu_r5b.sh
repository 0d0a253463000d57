# round 5: SQ counters of the sub-block blends (C) against the round-4 quadrant-pass blends (quadfwd, r04bwd)
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for v in C quadfwd r04bwd; do
  VARIANTS=$v bash tools/ab_pmc.sh || exit 1
  VARIANTS=$v PMC="SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_ANY SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH" bash tools/ab_pmc.sh || exit 1
done
