# round-4 call h: per-wave layout threshold (DI_WLONG_MIN) at 8.8 M docs, skewed and iid
O=gpurun_out/round4_h; mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal rc $1 in $2"; exit $1;; esac; }
for w in 512 128 64 32; do
  DI_WLONG_MIN=$w SWEEP=bm timeout -k 10 300 python3 tools/prune_sweep.py 8800000 skew > $O/sweep_bm_skew_w$w.json 2> $O/sweep_bm_skew_w$w.err; fatal $? skew_$w
done
for w in 512 128; do
  DI_WLONG_MIN=$w SWEEP=bm timeout -k 10 300 python3 tools/prune_sweep.py 8800000 > $O/sweep_bm_iid_w$w.json 2> $O/sweep_bm_iid_w$w.err; fatal $? iid_$w
  DI_WLONG_MIN=$w timeout -k 10 300 python3 bench.py --legs retrieve,retrieve_shard --steps 10 --warmup 2 --no-cpu > $O/bench_w$w.json 2> $O/bench_w$w.err; fatal $? bench_$w
done
echo all-done
