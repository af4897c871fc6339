#!/bin/bash
# candidate-workspace cap 1 GiB (ws1g, before) vs 4 GiB (new): retrieve legs same box,
# then exhaustive + block-max rows at 8.8 M skewed docs; scorer tests first
set -o pipefail
O=gpurun_out/round4_p8; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_index_gpu.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
VARIANTS="ws1g new ws1g new" bash tools/ab_scorer.sh round4_p8/ab 2>&1 | tee $O/ab.txt || exit 1
for v in ws1g new; do
  if [ $v = ws1g ]; then export DI_CAND_WS_MIB=1024; else unset DI_CAND_WS_MIB; fi
  SWEEP=bm timeout -k 10 400 python -u tools/prune_sweep.py 8800000 skew > $O/sweep_bm_$v.json 2> $O/sweep_bm_$v.err || { tail -5 $O/sweep_bm_$v.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/sweep_bm_$v.json').read().strip().splitlines()[-1])
print('$v', ' '.join('f%g:%.1fk' % (r['block_max_factor'], r['device_queries_per_s']/1e3) for r in d['rows']))"
done
