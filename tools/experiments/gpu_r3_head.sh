#!/bin/bash
# Round-3 HEAD: full GPU tier, 2-rank DP rehearsal, headline bench, headline kernel stats.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/gpu_suite.sh || exit 1
rm -rf gpurun_out/prof_head
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_head -o run -- python bench.py --steps 8 --warmup 3 > gpurun_out/prof_head.log 2>&1 || { tail -20 gpurun_out/prof_head.log; exit 1; }
find gpurun_out/prof_head -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} gpurun_out/kernel_stats_head.csv
rm -rf gpurun_out/prof_head
tail -1 gpurun_out/prof_head.log | cut -c1-200
