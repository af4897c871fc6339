#!/bin/bash
# sparse-item selection, setup-time posting count: scorer tests, same-box A/B of the
# retrieve legs (old = before, mid = the per-wave count at selection, new = setup count),
# then the 8.8 M skewed fixed-cost rows
set -o pipefail
O=gpurun_out/round4_p5; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_index_gpu.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
VARIANTS="old mid new old mid new" bash tools/ab_scorer.sh round4_p5/ab 2>&1 | tee $O/ab.txt || exit 1
for a in "128 skew 0" "32 skew 0"; do
  timeout -k 10 300 python -u tools/phase_prune.py 8800000 $a > "$O/phase_${a// /_}.txt" 2>&1 || exit $?
  tail -1 "$O/phase_${a// /_}.txt"
done
