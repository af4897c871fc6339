#!/bin/bash
# final call 1: the whole -m gpu suite, then smoke()
set -o pipefail
O=gpurun_out/${TAG:-round4_z}; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -5 $O/pytest_gpu.log; grep -E "FAILED|ERROR" $O/pytest_gpu.log | head -10; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1; rc=$?; tail -3 $O/smoke.log; exit $rc
