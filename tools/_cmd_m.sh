#!/bin/bash
# call m: block-max cost without skipping (factor 0.001) vs with, no block order; skewed 8.8 M
set -o pipefail
O=gpurun_out/round4_m; mkdir -p $O
fatal() { [ $1 -eq 0 ] || { echo "FAILED $2 rc=$1"; tail -5 $O/$2.txt; exit $1; }; }
run() {  # name ablate args...
  local n=$1 a=$2; shift 2
  DI_PROFILE_ABLATE=$a timeout -k 10 300 python3 tools/phase_prune.py 8800000 1 "$@" > $O/$n.txt 2>&1; fatal $? $n
  grep -q Traceback $O/$n.txt && exit 1
  echo "$n: $(tail -1 $O/$n.txt)"; grep "phase cycles" $O/$n.txt | tail -1
}
run skew_exh_ext 65600 skew 0
run skew_exh 64 skew 0
run skew_bm1_noskip_noorder 147520 skew 1
run skew_bm1_noorder 16448 skew 1
run skew_bm1_noskip_order 131136 skew 1
run skew_bm1_order 64 skew 1
