#!/bin/bash
# sparse-item selection: scorer GPU tests, then the 8.8 M skewed fixed-cost rows and the
# bench's retrieve legs (no regression on dense items)
set -o pipefail
O=gpurun_out/round4_p4; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_index_gpu.py -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log; grep -E "FAILED|Error" $O/pytest.log | head -5; [ $rc -eq 0 ] || exit $rc
for a in "128 skew 0" "32 skew 0" "8 skew 0" "1 skew 0"; do
  timeout -k 10 300 python -u tools/phase_prune.py 8800000 $a > "$O/phase_${a// /_}.txt" 2>&1 || exit $?
  tail -1 "$O/phase_${a// /_}.txt"
done
timeout -k 10 400 python3 -u bench.py --legs retrieve,retrieve_shard --steps 10 --warmup 2 --no-cpu > $O/bench_retrieve.json 2> $O/bench_retrieve.err || exit $?
python3 -c "
import json; d=json.loads(open('$O/bench_retrieve.json').read().strip().splitlines()[-1])
for l in ('retrieve','retrieve_shard'): print(l, d[l]['value'], d[l]['kernel_ms'])"
