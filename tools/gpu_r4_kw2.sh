#!/bin/bash
# gemm2s in-workgroup K-split (HSD_G2S_KW=2) : tests, then bench A/B at the small-batch configs (interleaved x2)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_gemm.py \
  -k "small_tiles or small_tt or dgrad_reading_w" > gpurun_out/kw2_tests.log 2>&1 || { tail -30 gpurun_out/kw2_tests.log; exit 1; }
tail -2 gpurun_out/kw2_tests.log
: > gpurun_out/kw2_ab.log
for r in 1 2; do
  for kw in 1 2; do
    HSD_G2S_KW=$kw timeout -k 10 300 python bench.py --model bert-large-uncased --seq_len 512 --batch_size 8 --steps 30 --warmup 5 2>/dev/null | tail -1 | cut -c1-150 | sed "s/^/bl8 kw=$kw /" >> gpurun_out/kw2_ab.log || exit 1
    HSD_G2S_KW=$kw timeout -k 10 300 python bench.py --batch_size 32 --steps 30 --warmup 5 2>/dev/null | tail -1 | cut -c1-150 | sed "s/^/bb32 kw=$kw /" >> gpurun_out/kw2_ab.log || exit 1
  done
done
cat gpurun_out/kw2_ab.log
