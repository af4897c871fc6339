#!/bin/bash
# A/B of one environment knob of the built library on bench legs, alternating on one box;
# one summary line per run (developer tool).
# Usage: VAR=DI_GEMM_STAGGER VALUES="0,0 48,0 0,0 48,0" LEGS=encode_x3 bash tools/ab_env.sh <tag>
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
tag=${1:-abenv}
mkdir -p "$R/gpurun_out/$tag"
i=0
for v in ${VALUES:?}; do
  i=$((i+1))
  out="$R/gpurun_out/$tag/run_$i"
  env "${VAR:?}=$v" timeout -k 10 ${RUN_TIMEOUT:-300} python3 "$R/bench.py" --steps ${STEPS:-3} \
    --warmup 1 --no-cpu --legs "${LEGS:-encode_x3}" > "$out.json" 2> "$out.err" || exit $?
  python3 - "$out.json" "$VAR=$v" <<'PY'
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
    for leg in ("retrieve", "retrieve_shard"):
        e = d.get(leg)
        if e:
            parts.append(f"{leg} {e['value']:.1f} {e.get('unit', '')}")
    print("  ".join(parts), flush=True)
PY
done
