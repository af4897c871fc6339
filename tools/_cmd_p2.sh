#!/bin/bash
# block-max dead-round sweep: scorer tests, then phase stamps at 8.8 M skewed docs
# (exhaustive, f = 1) and the fixed-cost ablations (min_impact 128, threshold off)
set -o pipefail
O=gpurun_out/round4_p2; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_index_gpu.py -x -q -k "block_max or packed or skew" --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for a in "1 skew 0" "1 skew 1" "128 skew 0"; do
  DI_PROFILE_ABLATE=64 timeout -k 10 300 python -u tools/phase_prune.py 8800000 $a > "$O/phase_${a// /_}.txt" 2>&1 || exit $?
  tail -2 "$O/phase_${a// /_}.txt"
done
DI_SCORE_THRESHOLD=0 DI_PROFILE_ABLATE=64 timeout -k 10 300 python -u tools/phase_prune.py 8800000 128 skew 0 > $O/phase_128_nothr.txt 2>&1 || exit $?
tail -2 $O/phase_128_nothr.txt
