#!/bin/bash
# The one GPU-box measurement entry point.  Steps run in order, each under its own time
# limit; the first failure ends the script.  Output under gpurun_out/$TAG.
#   STEPS (default "tests bench stats pmc"), space separated:
#   tests   pytest selection TESTS (default: the whole -m gpu suite)
#   bench   the default bench line (BENCH_ARGS) -> bench.json
#   ab      bench legs LEGS (default retrieve,retrieve_shard) per VARIANTS through
#           tools/ab_scorer.sh (old = tools/_old/libdeepimpact_hip.so, a baseline build)
#   encab   encode legs ENC_LEGS per VARIANTS through tools/ab_lib.sh
#   sweep   tools/prune_sweep.py SWEEP_ARGS (default "8800000 skew") with SWEEP
#           (default bm: exhaustive + block-max rows; exh: exhaustive only) per
#           SWEEP_VARIANTS (default new; old = the baseline build, ablate<N> = DI_PROFILE_ABLATE=N)
#   phases  scorer phase stamps (DI_PROFILE_ABLATE=PHASE_ABLATE, default 64) via
#           tools/phase_prune.py PHASE_ARGS
#   scorer_pmc  PMC passes (SCORER_PMC: counter groups split by '|') over
#           tools/phase_prune.py PHASE_ARGS -> spmc/summary.json
#   stats   rocprofv3 --kernel-trace --stats per leg, each leg ALONE (STAT_LEGS), so every
#           average in a CSV is that leg's -> stats_<leg>/run_kernel_stats.csv
#   pmc     PMC passes per leg (PMC_LEGS) through tools/pmc_legs.sh
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG=${TAG:-r5}
O="$R/gpurun_out/$TAG"
mkdir -p "$O"
OLD_ENV="DEEPIMPACT_HIP_LIB=$R/tools/_old/libdeepimpact_hip.so DI_LIB_ALLOW_MISSING=1"
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
    ab)
      (cd "$R" && VARIANTS="${VARIANTS:-old new old new}" bash tools/ab_scorer.sh "$TAG/ab" \
         "${LEGS:-retrieve,retrieve_shard}" 2>&1 | tee "$O/ab.txt") || exit 1 ;;
    encab)
      (cd "$R" && LEGS="${ENC_LEGS:-encode_x3}" VARIANTS="${VARIANTS:-old new old new}" \
         bash tools/ab_lib.sh "$TAG/encab" 2>&1 | tee "$O/encab.txt") || exit 1 ;;
    sweep)
      for v in ${SWEEP_VARIANTS:-new}; do
        n=$(echo "${SWEEP_ARGS:-8800000 skew}" | tr ' ' '_')
        case $v in old) E="$OLD_ENV" ;; ablate*) E="DI_PROFILE_ABLATE=${v#ablate}" ;;
          classes) E="DI_DEAL_CLASSES=1" ;;
          mid) E="DEEPIMPACT_HIP_LIB=$R/tools/_mid/libdeepimpact_hip.so DI_LIB_ALLOW_MISSING=1" ;;
          merge2) E="DI_PROFILE_MERGE=2" ;;
          mcap*) E="DI_MERGE_CAP=${v#mcap}" ;;
          *) E="X=0" ;; esac
        (cd "$R" && env $E SWEEP=${SWEEP:-bm} timeout -k 10 ${SWEEP_TIMEOUT:-500} python3 -u \
           tools/prune_sweep.py ${SWEEP_ARGS:-8800000 skew} > "$O/sweep_${n}_$v.json" \
           2> "$O/sweep_${n}_$v.err") || { tail -5 "$O/sweep_${n}_$v.err"; exit 1; }
        python3 - "$O/sweep_${n}_$v.json" "$v $n" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], " ".join(
    "m%d/f%g%s:%.1fk(r%.3f,merge %.1fms)" % (r["min_impact"], r["block_max_factor"], "p" if r["packed"] else "",
                               r["device_queries_per_s"] / 1e3, r["recall_at_1000"], r.get("merge_ms", -1))
    for r in d["rows"]), flush=True)
PY
      done ;;
    phases)
      (cd "$R" && DI_PROFILE_ABLATE=${PHASE_ABLATE:-64} timeout -k 10 ${PHASE_TIMEOUT:-500} python3 -u \
         tools/phase_prune.py ${PHASE_ARGS:-} > "$O/phases.txt" 2>&1)
      rc=$?; tail -20 "$O/phases.txt"; [ $rc -eq 0 ] || exit $rc ;;
    scorer_pmc)
      # PMC passes (one counter group each, --kernel-trace only) over tools/phase_prune.py
      # PHASE_ARGS; the synthetic collection is cached in /tmp between passes
      IFS='|' read -r -a GRPS <<< "${SCORER_PMC:-SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA|SQC_ICACHE_MISSES SQC_ICACHE_HITS SQ_IFETCH SQ_INSTS_VMEM SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VALU GRBM_GUI_ACTIVE}"
      i=0; mkdir -p "$O/spmc"
      for grp in "${GRPS[@]}"; do
        i=$((i+1))
        (cd /tmp && export TMPDIR=/tmp && SYNTH_CACHE=/tmp/di_synth timeout -k 10 ${PASS_TIMEOUT:-400} \
           rocprofv3 -M --pmc $grp --kernel-trace -d "$O/spmc/p$i" -o run --output-format csv -- \
           python3 "$R/tools/phase_prune.py" ${PHASE_ARGS:-8800000 128 skew} > "$O/spmc/p$i.txt" 2>&1)
        rc=$?; [ $rc -eq 0 ] || { tail -20 "$O/spmc/p$i.txt"; exit $rc; }
        echo "scorer pmc pass $i done"
      done
      python3 "$R/tools/pmc_summary.py" "$O/spmc" > "$O/spmc/summary.json" || exit 1 ;;
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
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
