#!/bin/bash
# TT weight gradient with one K-split accumulating in place (no fp32 atomics): tests, then roberta-large MLM A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_gemm.py tests/test_gpu_fp8.py \
  -k "tt or wgrad or mlm" > gpurun_out/ttdirect_tests.log 2>&1 || { tail -30 gpurun_out/ttdirect_tests.log; exit 1; }
tail -2 gpurun_out/ttdirect_tests.log
: > gpurun_out/ttdirect_ab.log
A="--model roberta-large --task masked-lm --seq_len 512 --batch_size 64 --steps 20 --warmup 5"
for r in 1 2; do
  for at in 0 1; do
    HSD_G2_TT_ATOMIC=$at timeout -k 10 300 python bench.py $A --dtype bf16 2>/dev/null | tail -1 | cut -c1-110 | sed "s/^/bf16 tt_atomic=$at /" >> gpurun_out/ttdirect_ab.log || exit 1
    HSD_G2_TT_ATOMIC=$at timeout -k 10 300 python bench.py $A --dtype fp8 2>/dev/null | tail -1 | cut -c1-110 | sed "s/^/fp8 tt_atomic=$at /" >> gpurun_out/ttdirect_ab.log || exit 1
  done
done
cat gpurun_out/ttdirect_ab.log
