#!/bin/bash
# PMC passes (counters with --kernel-trace only) over tools/attn_check for one mode.
# Usage: DI_ATTN=<mode> bash tools/pmc_attn.sh <tag>
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$R/gpurun_out/pmc_attn_${1:-run}"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC" \
           "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_BRANCH" \
           "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_FLAT"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 -M --pmc $grp --kernel-trace -d "$OUT/p$i" -o run --output-format csv \
     -- "$R/tools/attn_check" --nocheck > "$OUT/p$i.log" 2> "$OUT/p$i.err"
  rc=$?
  if [ $rc -ne 0 ]; then tail -20 "$OUT/p$i.err"; exit $rc; fi
done
python3 "$R/tools/pmc_summary.py" "$OUT" > "$OUT/summary.json"
python3 - "$OUT/summary.json" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))["kernels"]
for k, v in d.items():
    if "attention" in k:
        print(k, json.dumps({a: round(b, 1) for a, b in v.items()}, indent=0))
PY
