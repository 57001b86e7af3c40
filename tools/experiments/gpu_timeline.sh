#!/bin/bash
# rocprofv3 kernel trace of a short run; per-stream busy time and idle gaps of the last window.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/prof_tl
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_tl -o run -- python bench.py $BENCH_ARGS --steps 6 --warmup 3 > gpurun_out/prof_tl.log 2>&1 || { tail -20 gpurun_out/prof_tl.log; exit 1; }
f=$(find gpurun_out/prof_tl -name "*kernel_trace.csv" | head -1)
head -1 "$f"
python tools/timeline_gaps.py "$f" ${WINDOW_MS:-60}
rm -rf gpurun_out/prof_tl
