#!/bin/bash
# A/B of attention_x3 variants (DI_ATTN_X3 bits, launch_attention_x3: 0 = round-2 form,
# 4 = balanced query tiles, 8 = lazy max, 16 = interleaved softmax, 32 = two
# 4-wave workgroups per CU, 64 = three query tiles per wave; ":a" = DI_ATTN_X3_ABLATE a, timing only) on the bench's
# encode_x3 leg, one box, alternating; attention ms per step per run.
# Usage: VARIANTS="0 4 0:1 0:2 0:4" REPS=2 bash tools/ab_attn.sh
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$R/gpurun_out/ab_attn"
mkdir -p "$OUT"
for rep in $(seq 1 ${REPS:-2}); do
  for va in ${VARIANTS:-0 4}; do
    v=${va%%:*}; a=0; [ "$va" != "$v" ] && a=${va#*:}
    DI_ATTN_X3=$v DI_ATTN_X3_ABLATE=$a timeout -k 10 ${RUN_TIMEOUT:-240} python3 "$R/bench.py" --steps 3 --warmup 1 \
      --no-cpu --legs encode_x3 > "$OUT/v${v}a${a}_r${rep}.json" 2> "$OUT/v${v}a${a}_r${rep}.err" || exit $?
    python3 - "$OUT/v${v}a${a}_r${rep}.json" "$va" <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith("{"):
        d = json.loads(l)
        e = d.get("encode_fp32_faithful") or d
        k = e["kernels"]
        print(f"variant {sys.argv[2]}: {d['value']:.1f} docs/s attention {k['attention']['ms_per_step']:.2f} ms/step", flush=True)
PY
  done
done
