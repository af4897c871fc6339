# round-4 measurement call d: block-max / packed tests, attention_x3w parity + A/B,
# retrieve legs, configs[4] sweeps.  A failing test does not stop the data steps; a
# timeout, abort or crash (rc 124/134/137/139) stops everything.
O=gpurun_out/round4_d; mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal rc $1 in $2"; exit $1;; esac; }
timeout -k 10 600 python -u -m pytest tests/test_index_gpu.py -k "block_max or packed or skew" -m gpu -v -s --timeout 300 --timeout-method thread > $O/pytest_index.log 2>&1; rc=$?; tail -4 $O/pytest_index.log; fatal $rc index_tests
DI_ATTN_X3=64 timeout -k 10 600 python -u -m pytest tests/test_encoder_bf16x3_gpu.py tests/test_encoder_bert_gpu.py tests/test_encoder_phobert_gpu.py -m gpu -v -s --timeout 300 --timeout-method thread > $O/pytest_attn_x3w.log 2>&1; rc=$?; tail -4 $O/pytest_attn_x3w.log; fatal $rc attn_tests
timeout -k 10 300 python3 bench.py --legs encode_x3 --steps 5 --warmup 2 --no-cpu > $O/bench_x3_old.json 2> $O/bench_x3_old.err; fatal $? bench_old
DI_ATTN_X3=64 timeout -k 10 300 python3 bench.py --legs encode_x3 --steps 5 --warmup 2 --no-cpu > $O/bench_x3_new.json 2> $O/bench_x3_new.err; fatal $? bench_new
timeout -k 10 300 python3 bench.py --legs retrieve,retrieve_shard --no-cpu > $O/bench_retrieve.json 2> $O/bench_retrieve.err; fatal $? bench_retrieve
timeout -k 10 400 python3 tools/prune_sweep.py 8800000 skew > $O/sweep_8m_skew.json 2> $O/sweep_8m_skew.err; fatal $? sweep
SWEEP=bm DI_PROFILE_ABLATE=16384 timeout -k 10 300 python3 tools/prune_sweep.py 8800000 skew > $O/sweep_8m_skew_noorder.json 2> $O/sweep_8m_skew_noorder.err; fatal $? sweep_noorder
SWEEP=bm DI_PROFILE_ABLATE=24576 timeout -k 10 300 python3 tools/prune_sweep.py 8800000 skew > $O/sweep_8m_skew_nocoop.json 2> $O/sweep_8m_skew_nocoop.err; fatal $? sweep_nocoop
echo all-done
