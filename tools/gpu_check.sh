#!/bin/bash
# One GPU-box session: parity tests, a short bench, a rocprofv3 kernel-trace.
# Every GPU step has its own time limit; the first failure ends the script.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
mkdir -p gpurun_out
STEPS=${STEPS:-10}
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  timeout -k 10 900 python -m pytest tests -m gpu -x -q ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; tail -40 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
fi
if [ "${SKIP_BENCH:-0}" != "1" ]; then
  timeout -k 10 600 python bench.py --steps "$STEPS" --warmup 2 ${BENCH_ARGS:-} > gpurun_out/bench.json 2> gpurun_out/bench.err
  rc=$?; tail -5 gpurun_out/bench.err; cat gpurun_out/bench.json; [ $rc -eq 0 ] || exit $rc
fi
if [ "${PROFILE:-0}" = "1" ]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 600 rocprofv3 -M --kernel-trace --stats -d "$R/gpurun_out/prof" -o run --output-format csv \
     -- python3 "$R/bench.py" --steps 5 --warmup 1 --no-cpu ${BENCH_ARGS:-} > "$R/gpurun_out/prof_bench.json" 2> "$R/gpurun_out/prof.err"
  rc=$?; tail -5 "$R/gpurun_out/prof.err"; [ $rc -eq 0 ] || exit $rc
  find "$R/gpurun_out/prof" -name "*stats*" | head
fi
