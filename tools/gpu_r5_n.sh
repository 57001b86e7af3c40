#!/bin/bash
# Round 5 pass N: roberta-large MLM S=512 B=64 bf16 vs fp8 at HEAD (x2 interleaved) + fp8 kernel stats (no side stream)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/mlm_r5.log
for r in 1 2; do
  for dt in bf16 fp8; do
    timeout -k 10 400 python bench.py --steps 8 --warmup 3 --model roberta-large --task masked-lm --seq_len 512 --batch_size 64 --dtype $dt 2>/dev/null | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('roberta-large MLM B=64 $dt', d['value'], d['ms_per_step'])" | tee -a gpurun_out/mlm_r5.log || exit 1
  done
done
HSD_WGRAD_STREAM=0 PROF_NAME=r5_mlm_fp8_noside bash tools/prof_r4.sh --steps 4 --warmup 2 --model roberta-large --task masked-lm --seq_len 512 --batch_size 64 --dtype fp8 || exit 1
