#!/bin/bash
# weight-gradient plan for small steps: latency cost model (default) vs the fewest splits giving >= G workgroups
# (HSD_WGRAD_MIN_GRID), bert-large S=512 B=8 and bert-base B=32 / 64, interleaved x2
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
: > gpurun_out/mingrid.log
for r in 1 2; do
  for g in 0 128 192; do
    HSD_WGRAD_MIN_GRID=$g timeout -k 10 300 python bench.py --model bert-large-uncased --seq_len 512 --batch_size 8 --steps 30 --warmup 5 2>/dev/null | tail -1 | cut -c1-100 | sed "s/^/bl8 min_grid=$g /" >> gpurun_out/mingrid.log || exit 1
    HSD_WGRAD_MIN_GRID=$g timeout -k 10 300 python bench.py --batch_size 32 --steps 40 --warmup 5 2>/dev/null | tail -1 | cut -c1-100 | sed "s/^/bb32 min_grid=$g /" >> gpurun_out/mingrid.log || exit 1
    HSD_WGRAD_MIN_GRID=$g timeout -k 10 300 python bench.py --batch_size 64 --steps 30 --warmup 5 2>/dev/null | tail -1 | cut -c1-100 | sed "s/^/bb64 min_grid=$g /" >> gpurun_out/mingrid.log || exit 1
  done
done
cat gpurun_out/mingrid.log
