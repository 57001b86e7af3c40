#!/bin/bash
# Round-6 profiles: rocprofv3 kernel statistics of a bench config (PROF_ARGS) under tag PTAG, and optionally the fp8
# GEMM PMC passes (PMC8=1). Each GPU step has its own time limit; the first failure ends the script.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ -n "$PROF_ARGS" ]; then
  rm -rf gpurun_out/prof_${PTAG}
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${PTAG} -o run -- \
    python bench.py $PROF_ARGS > gpurun_out/prof_${PTAG}.log 2>&1 || { tail -20 gpurun_out/prof_${PTAG}.log; exit 1; }
  f=$(find gpurun_out/prof_${PTAG} -name "*kernel_stats.csv" | head -1)
  cp "$f" gpurun_out/kernel_stats_${PTAG}.csv
  tail -1 gpurun_out/prof_${PTAG}.log | cut -c1-200
  head -12 gpurun_out/kernel_stats_${PTAG}.csv | cut -c1-160
  rm -rf gpurun_out/prof_${PTAG}
fi
if [ -n "$PMC8" ]; then
  bash tools/pmc_gemm8.sh > gpurun_out/pmc_gemm8.log 2>&1 || { tail -20 gpurun_out/pmc_gemm8.log; exit 1; }
  cat gpurun_out/pmc_gemm8.tsv | cut -c1-150
  rm -rf gpurun_out/pmc8_*/
fi
