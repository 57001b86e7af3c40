#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
PROF_NAME=bl8b bash tools/prof_r4.sh --model bert-large-uncased --seq_len 512 --batch_size 8 --steps 20 --warmup 5 > gpurun_out/bl8b_summary.log 2>&1 || { tail -5 gpurun_out/bl8b_summary.log; exit 1; }
head -1 gpurun_out/bl8b_summary.log
python tools/trace_exclusive.py $(find gpurun_out/bl8b -name "*kernel_trace.csv" | head -1) 24
