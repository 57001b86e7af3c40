#!/bin/bash
# Round 5 GPU pass C: kernel stats of the headline and of the reference's literal fp32 config (bert-large S=512 B=8),
# the bf16 wire-cast cost, attention keep bits vs re-hashing at bert-large S=512 B=64, PMC of the dropout-residual GEMM.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
# per-kernel durations without the weight-gradient side stream (overlapping kernels inflate each other's durations)
HSD_WGRAD_STREAM=0 PROF_NAME=r5_head_noside bash tools/prof_r4.sh --steps 10 --warmup 3 || exit 1
HSD_WGRAD_STREAM=0 PROF_NAME=r5_fp32_bl8_noside bash tools/prof_r4.sh --model bert-large-uncased --seq_len 512 --batch_size 8 --dtype fp32 --steps 5 --warmup 2 || exit 1
timeout -k 10 600 python bench.py --model bert-large-uncased --seq_len 512 --batch_size 8 --dtype fp32 --steps 10 --warmup 3 > gpurun_out/bench_fp32.log 2>&1 || { tail -20 gpurun_out/bench_fp32.log; exit 1; }
tail -1 gpurun_out/bench_fp32.log | cut -c1-250
timeout -k 10 300 python tools/wire_cast_cost.py > gpurun_out/wire_cast_r5.jsonl 2>&1 || { tail -5 gpurun_out/wire_cast_r5.jsonl; exit 1; }
cat gpurun_out/wire_cast_r5.jsonl
: > gpurun_out/kmask_ab_r5.log
for r in 1 2; do
  for km in 1 0; do
    HSD_ATTN_KMASK=$km timeout -k 10 300 python bench.py --model bert-large-uncased --seq_len 512 --batch_size 64 --steps 8 --warmup 3 2>/dev/null | tail -1 | cut -c1-120 | sed "s/^/bl64 kmask=$km /" >> gpurun_out/kmask_ab_r5.log || exit 1
  done
done
cat gpurun_out/kmask_ab_r5.log
GEMMS="out_fwd_drop_res ffn2_fwd_drop_res ffn1_fwd_gelu_d ffn2_dgrad_mul_dbias" bash tools/pmc_r4_gemm.sh > gpurun_out/pmc_r5.log 2>&1 || { tail -5 gpurun_out/pmc_r5.log; exit 1; }
grep -E "VALU|MFMA|GRBM" gpurun_out/pmc4_summary.tsv
