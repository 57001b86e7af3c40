#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -3 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_ab_trees.sh 2 "head:--steps 20 --warmup 5" "bl8:--model bert-large-uncased --seq_len 512 --batch_size 8 --steps 30 --warmup 5" "bl64:--model bert-large-uncased --seq_len 512 --batch_size 64 --steps 8 --warmup 3"
