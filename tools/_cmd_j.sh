#!/bin/bash
# call j: query-sequential items (DI_SCORE_THRESHOLD=2) -- oracle test, then A/B on the retrieve legs
set -o pipefail
O=gpurun_out/round4_j; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_index_gpu.py -x -v --timeout 300 --timeout-method thread \
  -k "shared_threshold or block_max_exact or packed_postings_equal" > $O/pytest.log 2>&1; rc=$?; tail -8 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
VARIANTS="new thr2 thr1 new thr2 thr1" bash tools/ab_scorer.sh round4_j/ab retrieve,retrieve_shard || exit 1
