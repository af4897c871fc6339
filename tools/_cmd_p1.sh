#!/bin/bash
# phase stamps of the scorer at 8.8 M skewed docs: exhaustive, block-max f = 1, and the
# fixed cost (min_impact 128)
set -o pipefail
O=gpurun_out/round4_p1; mkdir -p $O
for a in "1 skew 0" "1 skew 1" "128 skew 0"; do
  DI_PROFILE_ABLATE=64 timeout -k 10 300 python -u tools/phase_prune.py 8800000 $a > "$O/phase_${a// /_}.txt" 2>&1 || exit $?
  tail -14 "$O/phase_${a// /_}.txt"
done
