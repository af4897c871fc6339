#!/bin/bash
# final call 4: configs[4] sweeps at 8.8 M docs (skewed and i.i.d.), every row
set -o pipefail
O=gpurun_out/round4_z; mkdir -p $O
timeout -k 10 540 python3 -u tools/prune_sweep.py 8800000 skew > $O/prune_sweep_skew.json 2> $O/prune_sweep_skew.err; rc=$?
tail -2 $O/prune_sweep_skew.err; [ $rc -eq 0 ] || exit $rc; grep -q Traceback $O/prune_sweep_skew.err && exit 1
timeout -k 10 540 python3 -u tools/prune_sweep.py 8800000 > $O/prune_sweep_iid.json 2> $O/prune_sweep_iid.err; rc=$?
tail -2 $O/prune_sweep_iid.err; [ $rc -eq 0 ] || exit $rc; grep -q Traceback $O/prune_sweep_iid.err && exit 1
echo done
