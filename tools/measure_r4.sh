#!/bin/bash
# Round-4 measurement call.  Steps (each with its own time limit; the first failure
# ends the script), selected by STEPS (default "tests bench stats pmc"):
#   tests  pytest selection TESTS (default: the whole -m gpu suite)
#   bench  the default bench line -> gpurun_out/$TAG/bench.json
#   stats  rocprofv3 --kernel-trace --stats per leg, each leg ALONE (STAT_LEGS), so every
#          average in a CSV is that leg's -> gpurun_out/$TAG/stats_<leg>/run_kernel_stats.csv
#   pmc    PMC passes per leg (PMC_LEGS) through tools/pmc_legs.sh
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG=${TAG:-r4}
O="$R/gpurun_out/$TAG"
mkdir -p "$O"
STEPS=${STEPS:-tests bench stats pmc}
for s in $STEPS; do
  case $s in
    tests)
      (cd "$R" && timeout -k 10 ${TEST_TIMEOUT:-900} python -u -m pytest ${TESTS:-tests -m gpu} -x -v \
         --timeout 300 --timeout-method thread > "$O/pytest_gpu.log" 2>&1)
      rc=$?; tail -15 "$O/pytest_gpu.log"; [ $rc -eq 0 ] || exit $rc ;;
    bench)
      (cd "$R" && timeout -k 10 ${BENCH_TIMEOUT:-600} python3 -u bench.py ${BENCH_ARGS:-} \
         > "$O/bench.json" 2> "$O/bench.err")
      rc=$?; tail -5 "$O/bench.err"; cat "$O/bench.json"; [ $rc -eq 0 ] || exit $rc ;;
    stats)
      for leg in ${STAT_LEGS:-encode_x3 retrieve retrieve_shard}; do
        (cd /tmp && export TMPDIR=/tmp && timeout -k 10 ${STAT_TIMEOUT:-400} rocprofv3 --kernel-trace --stats \
           -d "$O/stats_$leg" -o run --output-format csv -- \
           python3 "$R/bench.py" --legs "$leg" --steps ${STAT_STEPS:-5} --warmup 1 --no-cpu \
           > "$O/stats_$leg.json" 2> "$O/stats_$leg.err")
        rc=$?; [ $rc -eq 0 ] || { tail -20 "$O/stats_$leg.err"; exit $rc; }
        echo "stats $leg done"
      done ;;
    pmc)
      PMC_TAG=$TAG LEGS="${PMC_LEGS:-retrieve retrieve_shard}" \
        PMC_GROUPS="${PMC_GROUPS:-FETCH_SIZE|WRITE_SIZE|GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE TCC_HIT_sum TCC_MISS_sum}" \
        bash "$R/tools/pmc_legs.sh" || exit 1 ;;
  esac
done
