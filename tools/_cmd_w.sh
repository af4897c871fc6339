#!/bin/bash
# call w: the shared-threshold suffix sums as fixed-trip selects (no exec-masked loop)
set -o pipefail
O=gpurun_out/round4_w; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_index_gpu.py -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
VARIANTS="old new old new" bash tools/ab_scorer.sh round4_w/ab retrieve,retrieve_shard || exit 1
DI_PROFILE_ABLATE=64 timeout -k 10 300 python3 tools/phase_prune.py 1100000 1 > $O/phase_1100000.txt 2>&1 || exit 1
grep "phase cycles" $O/phase_1100000.txt | tail -1; tail -1 $O/phase_1100000.txt
