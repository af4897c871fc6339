#!/bin/bash
# A/B of the built library against tools/_old (and tools/_mid) libdeepimpact_hip.so (baseline builds)
# on bench legs, alternating on one box; one summary line per run.
# Usage: LEGS=encode_x3,encode VARIANTS="old new old new" bash tools/ab_lib.sh <tag>
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
tag=${1:-ablib}
mkdir -p "$R/gpurun_out/$tag"
i=0
for v in ${VARIANTS:-old new old new}; do
  i=$((i+1))
  out="$R/gpurun_out/$tag/${v}_$i"
  if [ "$v" = old ] || [ "$v" = mid ]; then  # baseline builds tools/_old, tools/_mid
    env DEEPIMPACT_HIP_LIB="$R/tools/_$v/libdeepimpact_hip.so" DI_LIB_ALLOW_MISSING=1 \
      timeout -k 10 ${RUN_TIMEOUT:-300} python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu \
      --legs "${LEGS:-encode_x3}" > "$out.json" 2> "$out.err" || exit $?
  else
    timeout -k 10 ${RUN_TIMEOUT:-300} python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu \
      --legs "${LEGS:-encode_x3}" > "$out.json" 2> "$out.err" || exit $?
  fi
  python3 - "$out.json" "$v" <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if not l.startswith("{"):
        continue
    d = json.loads(l)
    parts = [sys.argv[2]]
    for leg in ("encode_fp32_faithful", "encode_bf16"):
        e = d.get(leg)
        if e:
            k = e["kernels"]
            parts.append(f"{leg} {e['value']:.1f} docs/s " + " ".join(
                f"{n}={k[n]['ms_per_step']:.1f}" for n in ("gemm_qkv", "attention", "gemm_o", "gemm_ffn1", "gemm_ffn2"))
                + f" sha1={str(e.get('out_sha1'))[:10]}")
    print("  ".join(parts), flush=True)
PY
done
