#!/bin/bash
# A/B of encoder builds on the bench's encode_x3 leg (GPU box): the tools/_old library vs
# the in-tree one, alternating -> gpurun_out/<tag>_<variant>.json
set -o pipefail
tag=$1
run() {  # name, env...
    local name=$1; shift
    env "$@" timeout -k 10 300 python -u bench.py --legs encode_x3 --steps ${STEPS:-8} --warmup 2 --no-cpu \
        > gpurun_out/${tag}_${name}.json 2> gpurun_out/${tag}_${name}.err || return 1
    python3 - "$name" gpurun_out/${tag}_${name}.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
e = d["encode_fp32_faithful"]
k = {n: round(v["ms_per_step"], 2) for n, v in e["kernels"].items() if v["launches"]}
print(sys.argv[1], round(e["value"], 1), "docs/s", k, "sha1", e.get("out_sha1"), flush=True)
PY
}
for v in ${VARIANTS:-old new old new}; do
    case $v in
        old) run old DEEPIMPACT_HIP_LIB=$PWD/tools/_old/libdeepimpact_hip.so DI_LIB_ALLOW_MISSING=1 || exit 1 ;;
        mid) run mid DEEPIMPACT_HIP_LIB=$PWD/tools/_mid/libdeepimpact_hip.so DI_LIB_ALLOW_MISSING=1 || exit 1 ;;
        new) run new X=0 || exit 1 ;;
    esac
done
