#!/bin/bash
# call r: WLONG_MIN 128 (was 512) -- index tests, retrieve A/B, skewed 8.8 M sweep
set -o pipefail
O=gpurun_out/round4_r; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_index_gpu.py -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
VARIANTS="old new old new" bash tools/ab_scorer.sh round4_r/ab retrieve,retrieve_shard || exit 1
timeout -k 10 540 python3 -u tools/prune_sweep.py 8800000 skew > $O/prune_sweep_skew.json 2> $O/prune_sweep_skew.err; rc=$?
tail -2 $O/prune_sweep_skew.err; [ $rc -eq 0 ] || exit $rc; grep -q Traceback $O/prune_sweep_skew.err && exit 1
echo done
