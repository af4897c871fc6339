# round-4 call e: block-max (scalar threshold, block order, per-wave skipping) and packed
# (per-wave, small sublists plain) -- tests, retrieve legs, 8.8 M skewed sweeps + A/B
O=gpurun_out/round4_f; mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal rc $1 in $2"; exit $1;; esac; }
timeout -k 10 600 python -u -m pytest tests/test_index_gpu.py -m gpu -v -s --timeout 300 --timeout-method thread > $O/pytest_index.log 2>&1; rc=$?; tail -4 $O/pytest_index.log; fatal $rc index_tests
timeout -k 10 300 python3 bench.py --legs retrieve,retrieve_shard --no-cpu > $O/bench_retrieve.json 2> $O/bench_retrieve.err; fatal $? bench_retrieve
SWEEP=bm timeout -k 10 300 python3 tools/prune_sweep.py 8800000 skew > $O/sweep_bm.json 2> $O/sweep_bm.err; fatal $? sweep_bm
SWEEP=bm DI_PROFILE_ABLATE=32768 timeout -k 10 300 python3 tools/prune_sweep.py 8800000 skew > $O/sweep_bm_histq.json 2> $O/sweep_bm_histq.err; fatal $? sweep_histq
timeout -k 10 400 python3 tools/prune_sweep.py 8800000 skew > $O/sweep_8m_skew.json 2> $O/sweep_8m_skew.err; fatal $? sweep
timeout -k 10 400 python3 tools/prune_sweep.py 8800000 > $O/sweep_8m_iid.json 2> $O/sweep_8m_iid.err; fatal $? sweep_iid
echo all-done
DI_PROFILE_ABLATE=64 timeout -k 10 300 python3 tools/phase_prune.py 8800000 1 skew 0 > gpurun_out/round4_f/phase_skew_exh.txt 2>&1; fatal $? phase1
DI_PROFILE_ABLATE=64 timeout -k 10 300 python3 tools/phase_prune.py 8800000 1 skew 1 > gpurun_out/round4_f/phase_skew_bm1.txt 2>&1; fatal $? phase2
echo phases-done
