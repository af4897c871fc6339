#!/bin/bash
# final call 7: bench, per-leg stats (encode_x3, retrieve legs), encode PMC (traffic + busy split)
set -o pipefail
TAG=round4_z7 STEPS="bench stats pmc" STAT_LEGS="encode_x3 retrieve retrieve_shard" PMC_LEGS="encode_x3" bash tools/measure_r4.sh || exit 1
PASS_TIMEOUT=240 PMC_TAG=round4_z7b LEGS=encode_x3 \
  PMC_GROUPS="GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY|SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT" \
  bash tools/pmc_legs.sh || exit 1
echo done
