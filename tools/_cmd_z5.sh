#!/bin/bash
# final call 5 (WLONG_MIN 128): bench, per-leg stats, retrieve PMC, sweeps
set -o pipefail
TAG=round4_zz STEPS="bench stats pmc" STAT_LEGS="retrieve retrieve_shard" PMC_LEGS="retrieve retrieve_shard" bash tools/measure_r4.sh || exit 1
O=gpurun_out/round4_zz
timeout -k 10 500 python3 -u tools/prune_sweep.py 8800000 skew > $O/prune_sweep_skew.json 2> $O/prune_sweep_skew.err; rc=$?
tail -1 $O/prune_sweep_skew.err; [ $rc -eq 0 ] || exit $rc; grep -q Traceback $O/prune_sweep_skew.err && exit 1
timeout -k 10 500 python3 -u tools/prune_sweep.py 8800000 > $O/prune_sweep_iid.json 2> $O/prune_sweep_iid.err; rc=$?
tail -1 $O/prune_sweep_iid.err; [ $rc -eq 0 ] || exit $rc; grep -q Traceback $O/prune_sweep_iid.err && exit 1
echo done
