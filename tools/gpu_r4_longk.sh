#!/bin/bash
# long-K NT rule (256 x 256 kernel + K-splits for K >= 16384: the MLM head dgrad): tests + roberta-large MLM bench x2
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_gemm.py tests/test_gpu_fp8.py tests/test_gpu_e2e.py \
  -k "dgrad_reading_w or mlm or splitk or xent or cross_entropy" > gpurun_out/longk_tests.log 2>&1 || { tail -30 gpurun_out/longk_tests.log; exit 1; }
tail -2 gpurun_out/longk_tests.log
: > gpurun_out/longk_ab.log
A="--model roberta-large --task masked-lm --seq_len 512 --batch_size 64 --steps 20 --warmup 5"
for r in 1 2; do
  timeout -k 10 300 python bench.py $A --dtype bf16 2>/dev/null | tail -1 | cut -c1-110 | sed "s/^/bf16 /" >> gpurun_out/longk_ab.log || exit 1
  timeout -k 10 300 python bench.py $A --dtype fp8 2>/dev/null | tail -1 | cut -c1-110 | sed "s/^/fp8 /" >> gpurun_out/longk_ab.log || exit 1
done
cat gpurun_out/longk_ab.log
