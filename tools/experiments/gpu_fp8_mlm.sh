#!/bin/bash
# roberta-large MLM S=512: bf16 vs fp8 bench + fp8 kernel stats.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
B="--model roberta-large --task masked-lm --seq_len 512 --batch_size 64 --steps 10 --warmup 3"
for dt in bf16 fp8 bf16 fp8; do
  timeout -k 10 400 python bench.py $B --dtype $dt > gpurun_out/mlm_$dt.log 2>&1 || { tail -20 gpurun_out/mlm_$dt.log; exit 1; }
  echo "$dt $(tail -1 gpurun_out/mlm_$dt.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
rm -rf gpurun_out/prof_fp8
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_fp8 -o run -- python bench.py --model roberta-large --task masked-lm --seq_len 512 --batch_size 64 --steps 3 --warmup 2 --dtype fp8 > gpurun_out/prof_fp8.log 2>&1 || { tail -20 gpurun_out/prof_fp8.log; exit 1; }
find gpurun_out/prof_fp8 -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} gpurun_out/kernel_stats_fp8.csv
rm -rf gpurun_out/prof_fp8
head -25 gpurun_out/kernel_stats_fp8.csv | cut -d, -f1-5 | cut -c1-150
