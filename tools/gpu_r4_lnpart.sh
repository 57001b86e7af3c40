#!/bin/bash
# LayerNorm backward column partials (small row counts): tests, then bench A/B vs the per-block atomics
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ops.py tests/test_gpu_fp8.py \
  -k "ln or layer_norm or dense_residual or fused" > gpurun_out/lnpart_tests.log 2>&1 || { tail -30 gpurun_out/lnpart_tests.log; exit 1; }
tail -2 gpurun_out/lnpart_tests.log
: > gpurun_out/lnpart_ab.log
for r in 1 2; do
  for k in 32768 0; do
    HSD_LN_BWD_PART_ROWS=$k timeout -k 10 300 python bench.py --model bert-large-uncased --seq_len 512 --batch_size 8 --steps 30 --warmup 5 2>/dev/null | tail -1 | cut -c1-110 | sed "s/^/bl8 part_rows=$k /" >> gpurun_out/lnpart_ab.log || exit 1
    HSD_LN_BWD_PART_ROWS=$k timeout -k 10 300 python bench.py --batch_size 32 --steps 30 --warmup 5 2>/dev/null | tail -1 | cut -c1-110 | sed "s/^/bb32 part_rows=$k /" >> gpurun_out/lnpart_ab.log || exit 1
  done
done
cat gpurun_out/lnpart_ab.log
