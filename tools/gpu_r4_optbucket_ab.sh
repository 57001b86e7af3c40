#!/bin/bash
# optimizer-overlap slice size (HSD_OPT_BUCKET_MB) at bert-large S=512 B=8 and bert-base B=32, interleaved x2
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
: > gpurun_out/optbucket_ab.log
for r in 1 2; do
  for mb in ${MBS:-32 64 128}; do
    HSD_OPT_BUCKET_MB=$mb timeout -k 10 300 python bench.py --model bert-large-uncased --seq_len 512 --batch_size 8 --steps 30 --warmup 5 2>/dev/null | tail -1 | cut -c1-110 | sed "s/^/bl8 mb=$mb /" >> gpurun_out/optbucket_ab.log || exit 1
    HSD_OPT_BUCKET_MB=$mb timeout -k 10 300 python bench.py --batch_size 32 --steps 30 --warmup 5 2>/dev/null | tail -1 | cut -c1-110 | sed "s/^/bb32 mb=$mb /" >> gpurun_out/optbucket_ab.log || exit 1
  done
done
cat gpurun_out/optbucket_ab.log
