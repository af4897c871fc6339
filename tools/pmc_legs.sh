#!/bin/bash
# rocprofv3 PMC passes per bench leg (counters only with --kernel-trace, one counter
# group per pass, MI355X_MICROARCH.md's recipe), summarised per leg into
# gpurun_out/pmc_<TAG>/<leg>/summary.json (copy to profiles/<round>_pmc_<leg>.json:
# bench.py reads a leg's traffic from there).
# Usage: PMC_TAG=r02 LEGS="retrieve_shard encode_x3" bash tools/pmc_legs.sh
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG=${PMC_TAG:-run}
cd /tmp && export TMPDIR=/tmp
PMC_GRP_DEFAULT="FETCH_SIZE|WRITE_SIZE|GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT TCC_HIT_sum TCC_MISS_sum"
IFS='|' read -r -a PMC_GRPS <<< "${PMC_GROUPS:-$PMC_GRP_DEFAULT}"
for leg in ${LEGS:-retrieve_shard}; do
  OUT="$R/gpurun_out/pmc_$TAG/$leg"
  mkdir -p "$OUT"
  i=0
  for grp in "${PMC_GRPS[@]}"; do
    i=$((i+1))
    timeout -k 10 ${PASS_TIMEOUT:-300} rocprofv3 -M --pmc $grp --kernel-trace -d "$OUT/p$i" -o run \
       --output-format csv -- python3 "$R/bench.py" --steps 2 --warmup 1 --no-cpu --legs "$leg" \
       > "$OUT/p$i.json" 2> "$OUT/p$i.err"
    rc=$?
    if [ $rc -ne 0 ]; then tail -20 "$OUT/p$i.err"; exit $rc; fi
    echo "$leg pass $i done"
  done
  python3 "$R/tools/pmc_summary.py" "$OUT" > "$OUT/summary.json" || exit 1
done
