#!/bin/bash
# headline bench: weight gradients on the main stream (auto at B=1024) vs on the side stream (HSD_WGRAD_STREAM=1),
# interleaved x2
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
: > gpurun_out/side_ab.log
for r in 1 2; do
  for m in auto 1; do
    HSD_WGRAD_STREAM=$m timeout -k 10 300 python bench.py --steps 20 --warmup 5 2>/dev/null | tail -1 | cut -c1-160 | sed "s/^/wgrad_stream=$m /" >> gpurun_out/side_ab.log || exit 1
  done
done
cat gpurun_out/side_ab.log
