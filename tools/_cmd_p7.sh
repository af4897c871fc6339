#!/bin/bash
# final call: the whole GPU suite + smoke, the default bench, then the configs[4] sweeps
# with the pruned-search routing (EXT_BM for min_impact >= 16)
set -o pipefail
TAG=round4_p7 bash tools/_cmd_z1.sh || exit 1
TAG=round4_p7 STEPS="bench" bash tools/measure_r4.sh || exit 1
O=gpurun_out/round4_p7
for c in skew iid; do
  timeout -k 10 400 python -u tools/prune_sweep.py 8800000 $c > $O/prune_sweep_$c.json 2> $O/prune_sweep_$c.err || { tail -5 $O/prune_sweep_$c.err; exit 1; }
  echo "sweep $c done"
done
