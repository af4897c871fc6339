#!/bin/bash
# Round-3 measurement call: the default bench line, then rocprofv3 kernel stats of the
# headline leg (encode_x3 alone) and of the retrieve legs -- per-leg CSVs, so every
# average the bench reports is recomputable from one file.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG=${TAG:-r03k}
O="$R/gpurun_out"
timeout -k 10 900 python3 -u "$R/bench.py" > "$O/${TAG}_bench.json" 2> "$O/${TAG}_bench.err" || { tail -30 "$O/${TAG}_bench.err"; exit 1; }
echo "bench done"; tail -c 600 "$O/${TAG}_bench.json"
cd /tmp && export TMPDIR=/tmp
for leg in encode_x3 retrieve,retrieve_shard; do
  name=${leg//,/_}
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$O/${TAG}_prof_$name" -o run --output-format csv -- \
      python3 "$R/bench.py" --legs "$leg" --steps 5 --warmup 1 --no-cpu \
      > "$O/${TAG}_prof_$name.json" 2> "$O/${TAG}_prof_$name.err" || { tail -20 "$O/${TAG}_prof_$name.err"; exit 1; }
  echo "rocprof $leg done"
done
