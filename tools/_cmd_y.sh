#!/bin/bash
# call y: register-resident merge (merge_sel_kernel) -- index / sparse tests, then A/B
set -o pipefail
O=gpurun_out/round4_y; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_index_gpu.py tests/test_sparse_gpu.py tests/test_pipeline_gpu.py -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
VARIANTS="old new old new" bash tools/ab_scorer.sh round4_y/ab retrieve,retrieve_shard || exit 1
