#!/bin/bash
# One GPU-box measurement session: GPU parity tests, default bench, rocprofv3 kernel
# stats of a short bench, GEMM epilogue ablation sweep, scorer phase ablation.
# Every GPU step has its own time limit; the first failure ends the script.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
O="$R/gpurun_out/${TAG:-m}"
mkdir -p "$O"
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > "$O/pytest_gpu.log" 2>&1
  rc=$?; tail -5 "$O/pytest_gpu.log"; [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > "$O/bench.json" 2> "$O/bench.err"
rc=$?; tail -3 "$O/bench.err"; cat "$O/bench.json"; [ $rc -eq 0 ] || exit $rc
if [ "${PROFILE:-1}" = "1" ]; then
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$O/prof" \
     -o run --output-format csv -- python3 "$R/bench.py" --steps 5 --warmup 1 --no-cpu \
     > "$O/prof_bench.json" 2> "$O/prof.err")
  rc=$?; tail -3 "$O/prof.err"; [ $rc -eq 0 ] || exit $rc
fi
if [ "${GEMM:-1}" = "1" ] && [ -x tools/gemm_check ]; then
  timeout -k 10 300 tools/gemm_check --time > "$O/gemm_check.log" 2>&1
  rc=$?; grep -E "sweep|round 2" "$O/gemm_check.log"; [ $rc -eq 0 ] || exit $rc
fi
if [ "${ABLATE:-1}" = "1" ]; then
  for a in 0 1 2; do
    DI_PROFILE_ABLATE=$a timeout -k 10 300 python bench.py --legs retrieve --steps 5 --warmup 1 \
      --no-cpu > "$O/ablate_$a.json" 2>/dev/null || exit 1
    python3 -c "import json; d=json.load(open('$O/ablate_$a.json')); print('ablate $a', d['retrieve']['kernel_ms'])"
  done
fi
