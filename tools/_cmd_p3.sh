#!/bin/bash
# kernel split of the scorer's "score_blocks" time (item_setup vs score_blocks vs
# score_long) at 8.8 M skewed docs: exhaustive and min_impact 128
set -o pipefail
O=gpurun_out/round4_p3; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for a in "1 skew 0" "128 skew 0"; do
  d="$O/stats_${a// /_}"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$d" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/tools/phase_prune.py" 8800000 $a > "$GRAFT_REPO_ROOT/$d.txt" 2>&1 || exit $?
  tail -1 "$GRAFT_REPO_ROOT/$d.txt"
  cut -d, -f1-6 "$GRAFT_REPO_ROOT/$d/run_kernel_stats.csv" | cut -c1-160
done
