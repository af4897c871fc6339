#!/bin/bash
# sparse-item selection in the EXT_BM instantiation (pruned searches): scorer tests, then
# the configs[4] sweeps at 8.8 M docs (skewed and i.i.d.)
set -o pipefail
O=gpurun_out/round4_p6; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_index_gpu.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for c in skew iid; do
  timeout -k 10 400 python -u tools/prune_sweep.py 8800000 $c > $O/prune_sweep_$c.json 2> $O/prune_sweep_$c.err || { tail -5 $O/prune_sweep_$c.err; exit 1; }
  echo "sweep $c done"
done
