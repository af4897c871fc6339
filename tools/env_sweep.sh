#!/bin/bash
# Encode-leg timing for each value of one DI_* environment knob (A/B sweeps):
#   VAR=DI_GEMM_GM VALUES="4 8 16" bash tools/env_sweep.sh
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
O="$R/gpurun_out/${TAG:-env_sweep}"
mkdir -p "$O"
for v in ${VALUES:?}; do
  env "${VAR:?}=$v" timeout -k 10 300 python bench.py --legs ${LEGS:-encode} --steps 8 --warmup 2 \
    --no-cpu > "$O/s_$v.json" 2> "$O/s_$v.err" || exit 1
  python3 -c "import json; d=json.load(open('$O/s_$v.json')); e=d.get('encode',{}).get('kernels',{}); print('$VAR=$v', d['value'], {k: round(x['ms_per_step'],2) for k,x in e.items() if x['ms_per_step']>1})"
done
