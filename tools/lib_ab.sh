#!/bin/bash
# A/B of two builds of the library (DEEPIMPACT_HIP_LIB=$ALT, e.g. an experiment flag
# build) on the encode leg: bit-identity of per-token impacts and timing, alternated.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"
O="$R/gpurun_out/${TAG:-lib_ab}"
mkdir -p "$O"
ALT="$R/${ALT:?ALT=path/to/alt.so}"
timeout -k 10 300 python tools/encode_ab.py "$O/a.npy" > "$O/ab.log" 2>&1 || exit 1
DEEPIMPACT_HIP_LIB="$ALT" timeout -k 10 300 python tools/encode_ab.py "$O/b.npy" >> "$O/ab.log" 2>&1 || exit 1
python tools/encode_ab.py --compare "$O/a.npy" "$O/b.npy" | tee -a "$O/ab.log"
rm -f "$O/a.npy" "$O/b.npy"
for v in base alt base alt; do
  if [ $v = alt ]; then export DEEPIMPACT_HIP_LIB="$ALT"; else unset DEEPIMPACT_HIP_LIB; fi
  timeout -k 10 300 python bench.py --legs ${LEGS:-encode} --steps 8 --warmup 2 --no-cpu \
    > "$O/m_$v.json" 2> "$O/m_$v.err" || exit 1
  python3 -c "import json; d=json.load(open('$O/m_$v.json')); e=d.get('encode',{}).get('kernels',{}); print('$v', d['value'], {k: round(x['ms_per_step'],2) for k,x in e.items() if x['ms_per_step']>1})"
done
