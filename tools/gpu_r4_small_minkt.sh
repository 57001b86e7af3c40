#!/bin/bash
# one K-split for the weight gradients of small steps: bert-base B=32 (4,096 tokens) and B=64 (8,192) with the default
# plan vs HSD_WGRAD_MIN_KT = tokens / 64 (one split), interleaved x2
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
: > gpurun_out/small_minkt.log
for r in 1 2; do
  for k in 2 64; do
    HSD_WGRAD_MIN_KT=$k timeout -k 10 300 python bench.py --batch_size 32 --steps 30 --warmup 5 2>/dev/null | tail -1 | cut -c1-110 | sed "s/^/bb32 min_kt=$k /" >> gpurun_out/small_minkt.log || exit 1
  done
  for k in 2 128; do
    HSD_WGRAD_MIN_KT=$k timeout -k 10 300 python bench.py --batch_size 64 --steps 30 --warmup 5 2>/dev/null | tail -1 | cut -c1-110 | sed "s/^/bb64 min_kt=$k /" >> gpurun_out/small_minkt.log || exit 1
  done
  for k in 2 256; do
    HSD_WGRAD_MIN_KT=$k timeout -k 10 300 python bench.py --batch_size 128 --steps 20 --warmup 5 2>/dev/null | tail -1 | cut -c1-110 | sed "s/^/bb128 min_kt=$k /" >> gpurun_out/small_minkt.log || exit 1
  done
done
cat gpurun_out/small_minkt.log
