#!/bin/bash
# headline: weight-gradient K-splits with the side stream on -- default plan vs fewer splits (HSD_WGRAD_MIN_KT),
# interleaved x2
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
: > gpurun_out/minkt_ab.log
for r in 1 2; do
  for k in 2 256 700; do
    HSD_WGRAD_MIN_KT=$k timeout -k 10 300 python bench.py --steps 20 --warmup 5 2>/dev/null | tail -1 | cut -c1-110 | sed "s/^/min_kt=$k /" >> gpurun_out/minkt_ab.log || exit 1
  done
done
cat gpurun_out/minkt_ab.log
