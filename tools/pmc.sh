#!/bin/bash
# rocprofv3 PMC passes (counters only with --kernel-trace, one counter group per
# pass, as MI355X_MICROARCH.md prescribes) over a short bench run.
# Usage: PMC_TAG=r01 bash tools/pmc.sh [bench args...]
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG=${PMC_TAG:-run}
OUT="$R/gpurun_out/pmc_$TAG"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" \
           "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT" \
           "GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU TCC_HIT_sum TCC_MISS_sum" \
           "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_WAIT_INST_LDS SQ_INSTS_VMEM_WR SQ_LDS_UNALIGNED_STALL"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 -M --pmc $grp --kernel-trace -d "$OUT/p$i" -o run --output-format csv \
     -- python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu "$@" > "$OUT/p$i.json" 2> "$OUT/p$i.err"
  rc=$?
  if [ $rc -ne 0 ]; then tail -20 "$OUT/p$i.err"; exit $rc; fi
done
python3 "$R/tools/pmc_summary.py" "$OUT" > "$OUT/summary.json" && cat "$OUT/summary.json"
