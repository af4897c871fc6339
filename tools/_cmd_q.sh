#!/bin/bash
# call q: a 12-postings-per-lane scatter round (513..768 remaining: 768 slots, not 1024)
set -o pipefail
O=gpurun_out/round4_q; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_index_gpu.py -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
VARIANTS="old new old new" bash tools/ab_scorer.sh round4_q/ab retrieve,retrieve_shard || exit 1
