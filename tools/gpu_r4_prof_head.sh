#!/bin/bash
# headline kernel stats + exclusive (critical-path) time per kernel at HEAD
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
PROF_NAME=${PROF_NAME:-r4_head2} bash tools/prof_r4.sh --steps 10 --warmup 3 > gpurun_out/${PROF_NAME:-r4_head2}_summary.log 2>&1 || { tail -5 gpurun_out/${PROF_NAME:-r4_head2}_summary.log; exit 1; }
head -3 gpurun_out/${PROF_NAME:-r4_head2}_summary.log
python tools/trace_exclusive.py $(find gpurun_out/${PROF_NAME:-r4_head2} -name "*kernel_trace.csv" | head -1) 24
