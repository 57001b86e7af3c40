#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
: > gpurun_out/lnpart2_ab.log
for r in 1 2; do
  for cfg in "HSD_LN_BWD_PART_ROWS=0" "HSD_LN_BWD_PART_ROWS=32768 HSD_LN_BWD_PART_RPW=2" "HSD_LN_BWD_PART_ROWS=32768 HSD_LN_BWD_PART_RPW=4"; do
    env $cfg timeout -k 10 300 python bench.py --model bert-large-uncased --seq_len 512 --batch_size 8 --steps 30 --warmup 5 2>/dev/null | tail -1 | cut -c1-110 | sed "s/^/bl8 $cfg /" >> gpurun_out/lnpart2_ab.log || exit 1
  done
done
cat gpurun_out/lnpart2_ab.log
