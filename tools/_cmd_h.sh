# round-4 call h: per-wave layout threshold (DI_WLONG_MIN) at 8.8 M docs, skewed and iid
O=gpurun_out/round4_h; mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal rc $1 in $2"; exit $1;; esac; }
timeout -k 10 600 python -u -m pytest tests/test_index_gpu.py -k "block_max or packed or skew" -m gpu -v -s --timeout 300 --timeout-method thread > $O/pytest_index.log 2>&1; rc=$?; tail -3 $O/pytest_index.log; fatal $rc tests; [ $rc -eq 0 ] || exit 1
for w in 512 128 64 32; do
  DI_WLONG_MIN=$w SWEEP=bm timeout -k 10 300 python3 tools/prune_sweep.py 8800000 skew > $O/sweep_bm_skew_w$w.json 2> $O/sweep_bm_skew_w$w.err; fatal $? skew_$w; grep -q Traceback $O/sweep_bm_skew_w$w.err && exit 1
done
for w in 512 128; do
  DI_WLONG_MIN=$w SWEEP=bm timeout -k 10 300 python3 tools/prune_sweep.py 8800000 > $O/sweep_bm_iid_w$w.json 2> $O/sweep_bm_iid_w$w.err; fatal $? iid_$w
  DI_WLONG_MIN=$w timeout -k 10 300 python3 bench.py --legs retrieve,retrieve_shard --steps 10 --warmup 2 --no-cpu > $O/bench_w$w.json 2> $O/bench_w$w.err; fatal $? bench_$w
done
echo all-done
