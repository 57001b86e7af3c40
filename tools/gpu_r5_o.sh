#!/bin/bash
# Round 5 pass O: fp8 attention keep bits + fp8 out-projection dgrad delta rows; tests, roberta-large MLM fp8 A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_fp8.py tests/test_gpu_gemm.py -k "fp8 or q8 or row_dot or gemm8" -x -q --timeout 300 --timeout-method thread > gpurun_out/fp8_r5_tests.log 2>&1
rc=$?; tail -3 gpurun_out/fp8_r5_tests.log; [ $rc -eq 0 ] || exit $rc
: > gpurun_out/mlm_fp8_ab_r5.log
for r in 1 2; do
  for v in 0 1; do
    HSD_ATTN_KMASK=$v HSD_ATTN_DELTA_EPI=$v timeout -k 10 400 python bench.py --steps 8 --warmup 3 --model roberta-large --task masked-lm --seq_len 512 --batch_size 64 --dtype fp8 2>/dev/null | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('roberta-large MLM B=64 fp8 kmask+delta_epi=$v', d['value'], d['ms_per_step'])" | tee -a gpurun_out/mlm_fp8_ab_r5.log || exit 1
  done
done
