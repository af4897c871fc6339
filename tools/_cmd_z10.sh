#!/bin/bash
# final call 10: the whole GPU suite + smoke on the final tree, then the default bench and
# the retrieve legs' rocprof stats
set -o pipefail
TAG=round4_z10 bash tools/_cmd_z1.sh || exit 1
TAG=round4_z10 STEPS="bench stats" STAT_LEGS="retrieve retrieve_shard" bash tools/measure_r4.sh || exit 1
