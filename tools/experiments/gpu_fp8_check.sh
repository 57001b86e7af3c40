#!/bin/bash
# fp8 GEMM tests + roberta-large MLM S=512: fp8 (legacy vs persistent fp8 kernel) and bf16
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_fp8.py > gpurun_out/fp8_tests.log 2>&1 || { tail -30 gpurun_out/fp8_tests.log; exit 1; }
tail -1 gpurun_out/fp8_tests.log
R="--model roberta-large --task masked-lm --seq_len 512 --batch_size 64"
CONFIGS="$R --dtype fp8" bash tools/ab_env_bench.sh "HSD_G8_LEGACY=1" "HSD_G8_LEGACY=0" || exit 1
CONFIGS="$R --dtype bf16" bash tools/ab_env_bench.sh "HSD_G8_LEGACY=0" || exit 1
