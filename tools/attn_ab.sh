#!/bin/bash
# A/B of the attention v3 key loop (DI_ATTN_V3_MERGED=$MA vs $MB; 0 per-tile, 1 merged):
# bit-identity of the encoder's per-token impacts, GPU tests, encode-leg timing.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
O="$R/gpurun_out/${TAG:-attn_ab}"
MA=${MA:-0}; MB=${MB:-1}
mkdir -p "$O"
DI_ATTN_V3_MERGED=$MA timeout -k 10 300 python tools/encode_ab.py "$O/a.npy" > "$O/ab.log" 2>&1 || exit 1
DI_ATTN_V3_MERGED=$MB timeout -k 10 300 python tools/encode_ab.py "$O/b.npy" >> "$O/ab.log" 2>&1 || exit 1
python tools/encode_ab.py --compare "$O/a.npy" "$O/b.npy" | tee -a "$O/ab.log"
rm -f "$O/a.npy" "$O/b.npy"
DI_ATTN_V3_MERGED=$MB timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > "$O/pytest_gpu.log" 2>&1
rc=$?; tail -3 "$O/pytest_gpu.log"; [ $rc -eq 0 ] || exit $rc
for v in $MA $MB $MA $MB; do
  DI_ATTN_V3_MERGED=$v timeout -k 10 300 python bench.py --legs encode --steps 8 --warmup 2 --no-cpu \
    > "$O/m_$v.json" 2> "$O/m_$v.err" || exit 1
  python3 -c "import json; d=json.load(open('$O/m_$v.json')); e=d['encode']['kernels']; print('mode $v', d['value'], 'attention ms/step', round(e['attention']['ms_per_step'],2))"
done
