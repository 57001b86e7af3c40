#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
: > gpurun_out/attnS_batch_sweep.log
for b in 8 16 32 64; do
  ATTN_SHAPE=$b,512,16 timeout -k 10 120 python tools/attn_one.py 0.1 20 2>&1 | grep -v amdgpu.ids | sed "s/^/B=$b /" | tee -a gpurun_out/attnS_batch_sweep.log || exit 1
done
