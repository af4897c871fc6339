#!/bin/bash
# call n: VALU vs MFMA busy split of the encode kernels (attention_x3 first), two PMC passes
set -o pipefail
PASS_TIMEOUT=240 PMC_TAG=round4_n LEGS=encode_x3 \
  PMC_GROUPS="GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY|SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT" \
  bash tools/pmc_legs.sh || exit 1
python3 - <<'PY'
import json
d = json.load(open("gpurun_out/pmc_round4_n/encode_x3/summary.json"))
for k, v in d["kernels"].items():
    if any(s in k for s in ("attention", "gemm256")):
        print(k, {c: round(x, 1) for c, x in v.items()})
PY
