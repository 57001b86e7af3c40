#!/bin/bash
# Round 5 pass U: HEAD headline profile without the side stream + GEMM PMC (after the DMA-depth change)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
HSD_WGRAD_STREAM=0 PROF_NAME=r5_head_noside4 bash tools/prof_r4.sh --steps 10 --warmup 3 || exit 1
GEMMS="out_fwd_drop_res ffn2_fwd_drop_res ffn1_fwd_gelu_d ffn2_dgrad_mul_dbias" bash tools/pmc_r4_gemm.sh > gpurun_out/pmc_r5c.log 2>&1 || { tail -5 gpurun_out/pmc_r5c.log; exit 1; }
echo pmc ok
