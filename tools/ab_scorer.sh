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
for v in ${VARIANTS:-old new}; do
    case $v in
        old) run old DEEPIMPACT_HIP_LIB=$PWD/tools/_old/libdeepimpact_hip.so DI_LIB_ALLOW_MISSING=1 || exit 1 ;;
        mid) run mid DEEPIMPACT_HIP_LIB=$PWD/tools/_mid/libdeepimpact_hip.so DI_LIB_ALLOW_MISSING=1 || exit 1 ;;
        new) run new X=0 || exit 1 ;;
        ws1g) run ws1g DI_CAND_WS_MIB=1024 || exit 1 ;;
        ablate*) run $v DI_PROFILE_ABLATE=${v#ablate} || exit 1 ;;
        wlong*) run $v DI_WLONG_MIN=${v#wlong} || exit 1 ;;
        b32) run $v DI_PROFILE_ABLATE=4096 DI_DEAL_X4=0 || exit 1 ;;  # 4-byte loads, 32-block dealing
        x4deal32) run $v DI_DEAL_X4=0 || exit 1 ;;                    # 16-byte loads, 32-block dealing
        classes) run $v DI_DEAL_CLASSES=1 || exit 1 ;;                # one class-ordered posting array
        nohs) run $v DI_PROFILE_ABLATE=1048576 || exit 1 ;;           # no histogram-area staging
        noemit) run $v DI_PROFILE_ABLATE=2097152 || exit 1 ;;         # no few-block emit-above
        mcap*) run $v DI_MERGE_CAP=${v#mcap} || exit 1 ;;              # merge LDS key capacity
    esac
done
