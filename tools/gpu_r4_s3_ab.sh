#!/bin/bash
# 128 x 128 GEMMs: stage count rule (3 stages + 8 waves only for one-round grids) vs 3 stages (8-wave K-split) for
# every gemm2s grid (HSD_G2S_STAGES=3), bert-large S=512 B=8 and bert-base B=32, interleaved x2
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
: > gpurun_out/s3_ab.log
for r in 1 2; do
  for s in auto 3; do
    if [ $s = auto ]; then E=""; else E="HSD_G2S_STAGES=3"; fi
    env $E timeout -k 10 300 python bench.py --model bert-large-uncased --seq_len 512 --batch_size 8 --steps 30 --warmup 5 2>/dev/null | tail -1 | cut -c1-110 | sed "s/^/bl8 stages=$s /" >> gpurun_out/s3_ab.log || exit 1
    env $E timeout -k 10 300 python bench.py --batch_size 32 --steps 30 --warmup 5 2>/dev/null | tail -1 | cut -c1-110 | sed "s/^/bb32 stages=$s /" >> gpurun_out/s3_ab.log || exit 1
  done
done
cat gpurun_out/s3_ab.log
