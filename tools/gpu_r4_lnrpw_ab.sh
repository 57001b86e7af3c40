#!/bin/bash
# LayerNorm backward rows per wave floor (HSD_LN_BWD_MIN_RPW) at bert-large S=512 B=8, interleaved x2
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
: > gpurun_out/lnrpw_ab.log
for r in 1 2; do
  for k in 4 2 8 16; do
    HSD_LN_BWD_MIN_RPW=$k timeout -k 10 300 python bench.py --model bert-large-uncased --seq_len 512 --batch_size 8 --steps 30 --warmup 5 2>/dev/null | tail -1 | cut -c1-110 | sed "s/^/bl8 min_rpw=$k /" >> gpurun_out/lnrpw_ab.log || exit 1
  done
done
cat gpurun_out/lnrpw_ab.log
