#!/bin/bash
# optimizer-overlap slice size 32 vs 16 MiB at the headline (bert-base B=1024) and bert-large S=512 B=8, interleaved x2
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
: > gpurun_out/optbucket2_ab.log
for r in 1 2; do
  for mb in 32 16; do
    HSD_OPT_BUCKET_MB=$mb timeout -k 10 300 python bench.py --steps 20 --warmup 5 2>/dev/null | tail -1 | cut -c1-110 | sed "s/^/bb1024 mb=$mb /" >> gpurun_out/optbucket2_ab.log || exit 1
    HSD_OPT_BUCKET_MB=$mb timeout -k 10 300 python bench.py --model bert-large-uncased --seq_len 512 --batch_size 8 --steps 30 --warmup 5 2>/dev/null | tail -1 | cut -c1-110 | sed "s/^/bl8 mb=$mb /" >> gpurun_out/optbucket2_ab.log || exit 1
  done
done
cat gpurun_out/optbucket2_ab.log
