set -o pipefail
O=gpurun_out/round4_d; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_index_gpu.py -k "block_max or packed or skew" -m gpu -x -v -s --timeout 300 --timeout-method thread > $O/pytest_index.log 2>&1; rc=$?; tail -5 $O/pytest_index.log; [ $rc -eq 0 ] || exit $rc
DI_ATTN_X3=64 timeout -k 10 600 python -u -m pytest tests/test_encoder_bf16x3_gpu.py tests/test_encoder_bert_gpu.py tests/test_encoder_phobert_gpu.py -m gpu -x -v -s --timeout 300 --timeout-method thread > $O/pytest_attn_x3w.log 2>&1; rc=$?; tail -5 $O/pytest_attn_x3w.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench.py --legs encode_x3 --steps 5 --warmup 2 --no-cpu > $O/bench_x3_old.json 2> $O/bench_x3_old.err || exit 1
DI_ATTN_X3=64 timeout -k 10 300 python3 bench.py --legs encode_x3 --steps 5 --warmup 2 --no-cpu > $O/bench_x3_new.json 2> $O/bench_x3_new.err || exit 1
timeout -k 10 300 python3 bench.py --legs retrieve,retrieve_shard --no-cpu > $O/bench_retrieve.json 2> $O/bench_retrieve.err || exit 1
timeout -k 10 400 python3 tools/prune_sweep.py 8800000 skew > $O/sweep_8m_skew.json 2> $O/sweep_8m_skew.err || exit 1
SWEEP=bm DI_PROFILE_ABLATE=8192 timeout -k 10 300 python3 tools/prune_sweep.py 8800000 skew > $O/sweep_8m_skew_nocoop.json 2> $O/sweep_8m_skew_nocoop.err
