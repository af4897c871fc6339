#!/bin/bash
# call t: attention_x3 -- one branch per fragment-read site (AX_SEL over b, u constant)
set -o pipefail
O=gpurun_out/round4_t; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_encoder_bf16x3_gpu.py tests/test_encoder_phobert_gpu.py tests/test_encoder_bert_gpu.py -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
bash tools/ab_encode.sh round4_t/ab || exit 1
