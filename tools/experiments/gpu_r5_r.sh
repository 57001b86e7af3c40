#!/bin/bash
# Round 5 pass R: fp32 linear layers from one read of each operand (split3x2 + fused bias-gradient column sums)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_fp32.py -x -q --timeout 300 --timeout-method thread > gpurun_out/fp32_r_tests.log 2>&1
rc=$?; tail -3 gpurun_out/fp32_r_tests.log; [ $rc -eq 0 ] || exit $rc
: > gpurun_out/fp32_r.log
for r in 1 2; do
  timeout -k 10 400 python bench.py --model bert-large-uncased --seq_len 512 --batch_size 8 --dtype fp32 --steps 10 --warmup 3 2>/dev/null | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('fp32 bert-large B=8 split3x2', d['value'], d['ms_per_step'])" | tee -a gpurun_out/fp32_r.log || exit 1
done
HSD_WGRAD_STREAM=0 PROF_NAME=r5_fp32_bl8_x2 bash tools/prof_r4.sh --model bert-large-uncased --seq_len 512 --batch_size 8 --dtype fp32 --steps 5 --warmup 2 || exit 1
