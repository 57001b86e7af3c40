#!/bin/bash
# bert-large S=512 B=8: NT tile choice with the 8-wave gemm2s: default (256 tiles above 128 big tiles) vs 128 x 128
# everywhere (2 stages, 2 workgroups per CU) vs 128 x 128 everywhere with 3 stages (8-wave K-split, 1 per CU)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
: > gpurun_out/small_ab.log
A="--model bert-large-uncased --seq_len 512 --batch_size 8 --steps 30 --warmup 5"
for r in 1 2; do
  timeout -k 10 300 python bench.py $A 2>/dev/null | tail -1 | cut -c1-120 | sed "s/^/default /" >> gpurun_out/small_ab.log || exit 1
  HSD_G2_SMALL=1 timeout -k 10 300 python bench.py $A 2>/dev/null | tail -1 | cut -c1-120 | sed "s/^/small /" >> gpurun_out/small_ab.log || exit 1
  HSD_G2_SMALL=1 HSD_G2S_STAGES=3 timeout -k 10 300 python bench.py $A 2>/dev/null | tail -1 | cut -c1-120 | sed "s/^/small_s3 /" >> gpurun_out/small_ab.log || exit 1
done
cat gpurun_out/small_ab.log
