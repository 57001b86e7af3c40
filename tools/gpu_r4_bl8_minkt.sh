#!/bin/bash
# weight-gradient minimum K-tiles per split (HSD_WGRAD_MIN_KT) at bert-large S=512 B=8, interleaved x2
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
: > gpurun_out/bl8_minkt.log
for r in 1 2; do
  for k in ${KS:-2 4 8 16}; do
    HSD_WGRAD_MIN_KT=$k timeout -k 10 300 python bench.py --model bert-large-uncased --seq_len 512 --batch_size 8 --steps 30 --warmup 5 2>/dev/null | tail -1 | cut -c1-110 | sed "s/^/bl8 min_kt=$k /" >> gpurun_out/bl8_minkt.log || exit 1
  done
done
cat gpurun_out/bl8_minkt.log
