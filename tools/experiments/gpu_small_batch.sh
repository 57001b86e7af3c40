#!/bin/bash
# The reference's own per-rank config (bert-large-wwm, B = 8, S = 512): tests of the small-step paths, A/B of the
# stored Wᵀ (HSD_WT=1) vs the W-direct dgrads (HSD_WT=0), interleaved, then a kernel-trace profile.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_gemm.py tests/test_gpu_e2e.py -x -q --timeout 300 --timeout-method thread -k "directly or without_stored or cls or dgrad or fp32_mode" > gpurun_out/small_tests.log 2>&1
rc=$?; tail -4 gpurun_out/small_tests.log; [ $rc -eq 0 ] || exit $rc
B="--model bert-large-uncased-whole-word-masking --seq_len 512 --batch_size 8 --steps 30 --warmup 5"
: > gpurun_out/small_ab.log
for r in 1 2; do
  for wt in 1 0; do
    HSD_WT=$wt timeout -k 10 300 python bench.py $B > gpurun_out/small_one.log 2>&1 || { tail -20 gpurun_out/small_one.log; exit 1; }
    echo "HSD_WT=$wt $(tail -1 gpurun_out/small_one.log | cut -c1-200)" | tee -a gpurun_out/small_ab.log
  done
done
rm -rf gpurun_out/prof_small
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_small -o run -- python bench.py $B > gpurun_out/prof_small.log 2>&1 || { tail -20 gpurun_out/prof_small.log; exit 1; }
find gpurun_out/prof_small -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} gpurun_out/kernel_stats_small.csv
head -25 gpurun_out/kernel_stats_small.csv | cut -d, -f1-4 | cut -c1-160
