#!/bin/bash
# MLM head on the hand GEMMs: numerics test, roberta-large MLM bench (bf16), kernel trace (library GEMMs must be gone).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py -x -q --timeout 300 --timeout-method thread -k "mlm or cls or xent or cross" > gpurun_out/mlm_tests.log 2>&1
rc=$?; tail -4 gpurun_out/mlm_tests.log; [ $rc -eq 0 ] || exit $rc
B="--model roberta-large --task masked-lm --seq_len 512 --batch_size 64 --steps 10 --warmup 3"
timeout -k 10 400 python bench.py $B > gpurun_out/mlm_bench.log 2>&1 || { tail -20 gpurun_out/mlm_bench.log; exit 1; }
tail -1 gpurun_out/mlm_bench.log | cut -c1-330
rm -rf gpurun_out/prof_mlm
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_mlm -o run -- python bench.py --model roberta-large --task masked-lm --seq_len 512 --batch_size 64 --steps 3 --warmup 2 > gpurun_out/prof_mlm.log 2>&1 || { tail -20 gpurun_out/prof_mlm.log; exit 1; }
find gpurun_out/prof_mlm -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} gpurun_out/kernel_stats_mlm.csv
grep -c "Cijk" gpurun_out/kernel_stats_mlm.csv || true
