#!/bin/bash
# call s: attention_x3 -- the full sub-chunk skips the key mask (uniform branch)
set -o pipefail
O=gpurun_out/round4_s; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_encoder_bf16x3_gpu.py tests/test_encoder_phobert_gpu.py tests/test_encoder_bert_gpu.py -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
bash tools/ab_encode.sh round4_s/ab || exit 1
