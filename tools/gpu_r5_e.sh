#!/bin/bash
# Round 5 pass E: GPU tier after the attention / GELU changes, attention timings, headline batch sweep
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -3 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
{ timeout -k 10 120 python tools/attn_one.py 0.1 20 && ATTN_SHAPE=64,512,16 timeout -k 10 120 python tools/attn_one.py 0.1 20 &&
  ATTN_KMASK=0 ATTN_SHAPE=64,512,16 timeout -k 10 120 python tools/attn_one.py 0.1 20; } 2>&1 | grep -v amdgpu.ids | tee gpurun_out/attn_r5e.log || exit 1
: > gpurun_out/batch_sweep_r5.log
for b in 1024 1280 1536 768 1024; do
  for ws in auto 1; do
    HSD_WGRAD_STREAM=$ws timeout -k 10 300 python bench.py --batch_size $b --steps 12 --warmup 4 2>/dev/null | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('B=$b wgrad_stream=$ws', d['value'], d['ms_per_step'])" | tee -a gpurun_out/batch_sweep_r5.log || exit 1
  done
done
