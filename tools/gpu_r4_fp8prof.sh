#!/bin/bash
# HEAD fp8 evidence: roberta-large MLM S=512 B=64 kernel stats in bf16 and fp8 (calibrated steps: no quant_kernel)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
for dt in fp8 bf16; do
  PROF_NAME=mlm_$dt bash tools/prof_r4.sh --model roberta-large --task masked-lm --seq_len 512 --batch_size 64 --dtype $dt --steps 10 --warmup 5 || exit 1
  grep -c "quant_kernel\|amax_kernel" gpurun_out/kernel_stats_mlm_$dt.csv || true
done
