#!/bin/bash
# after the 4 GiB candidate workspace (one launch per step at 1.1 M docs): PMC of the
# retrieve_shard leg re-collected (copied to profiles/ so the bench line reads it), the
# default bench, then the GPU suite + smoke
set -o pipefail
PMC_TAG=round4_zzz LEGS="retrieve_shard" \
  PMC_GROUPS="FETCH_SIZE|WRITE_SIZE|GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE TCC_HIT_sum TCC_MISS_sum" \
  bash tools/pmc_legs.sh || exit 1
cp gpurun_out/pmc_round4_zzz/retrieve_shard/summary.json profiles/round4_zzz_pmc_retrieve_shard.json || exit 1
mkdir -p gpurun_out/round4_p9 && cp profiles/round4_zzz_pmc_retrieve_shard.json gpurun_out/round4_p9/
TAG=round4_p9 STEPS="bench" bash tools/measure_r4.sh || exit 1
# (the GPU suite: the round-end driver run)
