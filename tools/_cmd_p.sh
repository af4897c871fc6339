#!/bin/bash
# call p: per-wave scatter imbalance (wave-mean scatter vs the scatter phase of workgroup 0)
set -o pipefail
O=gpurun_out/round4_p; mkdir -p $O
for n in 100000 1100000; do
  DI_PROFILE_ABLATE=64 timeout -k 10 300 python3 tools/phase_prune.py $n 1 > $O/phase_$n.txt 2>&1 || { tail -5 $O/phase_$n.txt; exit 1; }
  grep -q Traceback $O/phase_$n.txt && exit 1
  echo "$n: $(tail -1 $O/phase_$n.txt)"; grep "phase cycles" $O/phase_$n.txt | tail -1
done
