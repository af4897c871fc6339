#!/bin/bash
# call o: wave_append<MB> only in the block-max / packed instantiations (the plain scorer's
# code is unchanged), tqn last in ScoreShared; index tests, then skewed/iid 8.8 M phases
set -o pipefail
O=gpurun_out/round4_o; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_index_gpu.py -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
fatal() { [ $1 -eq 0 ] || { echo "FAILED $2 rc=$1"; tail -5 $O/$2.txt; exit $1; }; }
run() {  # name ablate args...
  local n=$1 a=$2; shift 2
  DI_PROFILE_ABLATE=$a timeout -k 10 300 python3 tools/phase_prune.py 8800000 1 "$@" > $O/$n.txt 2>&1; fatal $? $n
  grep -q Traceback $O/$n.txt && exit 1
  echo "$n: $(tail -1 $O/$n.txt)"; grep "phase cycles" $O/$n.txt | tail -1
}
run skew_exh 64 skew 0
run skew_exh_ext 65600 skew 0
run skew_bm1 64 skew 1
run skew_bm1_noorder 16448 skew 1
run iid_exh 64 iid 0
run iid_bm1 64 iid 1
run iid_bm1_noorder 16448 iid 1
