#!/bin/bash
# call y2: the register merge also for lists whose total may pass its registers (flagged queries
# to the general kernel) -- index / sparse / multirank tests, then A/B
set -o pipefail
O=gpurun_out/round4_y2; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests/test_index_gpu.py tests/test_sparse_gpu.py tests/test_multirank_gpu.py -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
VARIANTS="old new old new" bash tools/ab_scorer.sh round4_y2/ab retrieve,retrieve_shard || exit 1
