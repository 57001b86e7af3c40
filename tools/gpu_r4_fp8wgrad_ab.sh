#!/bin/bash
# roberta-large MLM S=512 B=64: bf16 vs fp8 (bf16 weight gradients, HSD_FP8_WGRAD=0) vs fp8 (fp8 weight gradients),
# interleaved x2, then the fp8 step's kernel stats
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
A="--model roberta-large --task masked-lm --seq_len 512 --batch_size 64 --steps 20 --warmup 5"
: > gpurun_out/fp8wgrad_ab.log
for r in 1 2; do
  timeout -k 10 300 python bench.py $A --dtype bf16 2>/dev/null | tail -1 | sed "s/^/bf16 /" >> gpurun_out/fp8wgrad_ab.log || exit 1
  HSD_FP8_WGRAD=0 timeout -k 10 300 python bench.py $A --dtype fp8 2>/dev/null | tail -1 | sed "s/^/fp8_bf16wgrad /" >> gpurun_out/fp8wgrad_ab.log || exit 1
  timeout -k 10 300 python bench.py $A --dtype fp8 2>/dev/null | tail -1 | sed "s/^/fp8_fp8wgrad /" >> gpurun_out/fp8wgrad_ab.log || exit 1
done
cut -c1-140 gpurun_out/fp8wgrad_ab.log
PROF_NAME=mlm_fp8w bash tools/prof_r4.sh --model roberta-large --task masked-lm --seq_len 512 --batch_size 64 --dtype fp8 --steps 10 --warmup 5 > /dev/null 2>&1 || exit 1
head -14 gpurun_out/kernel_stats_mlm_fp8w.csv | cut -c1-120
