#!/bin/bash
# A/B of scorer builds / profiling ablations on the retrieve legs (GPU box).
# usage: tools/ab_scorer.sh <tag> [legs]   -> gpurun_out/<tag>_<variant>.json
set -o pipefail
tag=$1; legs=${2:-retrieve,retrieve_shard}
run() {  # name, env...
    local name=$1; shift
    env "$@" timeout -k 10 240 python -u bench.py --legs "$legs" --steps 10 --warmup 2 --no-cpu \
        > gpurun_out/${tag}_${name}.json 2> gpurun_out/${tag}_${name}.err || return 1
    python3 - "$name" gpurun_out/${tag}_${name}.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
out = [sys.argv[1]]
for k in ("retrieve", "retrieve_shard", "retrieve_full"):
    if k in d:
        out.append(f"{k}: {d[k]['value']:.0f} q/s score_blocks {d[k]['kernel_ms']['score_blocks']:.3f} ms/launch")
print("  ".join(out), flush=True)
PY
}
run old DEEPIMPACT_HIP_LIB=$PWD/tools/_old/libdeepimpact_hip.so || exit 1
run new X=0 || exit 1
run nokey DI_PROFILE_ABLATE=2048 || exit 1
run rw DI_PROFILE_ABLATE=4096 || exit 1
run rw_nokey DI_PROFILE_ABLATE=6144 || exit 1
run noscatter DI_PROFILE_ABLATE=1 || exit 1
