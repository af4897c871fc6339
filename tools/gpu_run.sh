#!/bin/bash
# One GPU-box session: pytest selection (TESTS, default the whole -m gpu suite), a
# bench run (BENCH_ARGS; SKIP_BENCH=1 skips), optionally a rocprofv3 kernel-trace of a
# short bench (PROFILE=1).  Every GPU step has its own time limit; the first failure
# ends the script.  Output under gpurun_out/$TAG.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
O="$R/gpurun_out/${TAG:-run}"
mkdir -p "$O"
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  timeout -k 10 ${TEST_TIMEOUT:-600} python -u -m pytest ${TESTS:-tests -m gpu} -x -v -s \
    --timeout 300 --timeout-method thread > "$O/pytest_gpu.log" 2>&1
  rc=$?; tail -15 "$O/pytest_gpu.log"; [ $rc -eq 0 ] || exit $rc
fi
if [ "${SKIP_BENCH:-0}" != "1" ]; then
  timeout -k 10 ${BENCH_TIMEOUT:-600} python bench.py ${BENCH_ARGS:-} > "$O/bench.json" 2> "$O/bench.err"
  rc=$?; tail -5 "$O/bench.err"; cat "$O/bench.json"; [ $rc -eq 0 ] || exit $rc
fi
if [ "${PROFILE:-0}" = "1" ]; then
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$O/prof" \
     -o run --output-format csv -- python3 "$R/bench.py" --steps 5 --warmup 1 --no-cpu ${PROF_ARGS:-} \
     > "$O/prof_bench.json" 2> "$O/prof.err")
  rc=$?; tail -3 "$O/prof.err"; [ $rc -eq 0 ] || exit $rc
fi
