#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_fp8.py -x -q -m gpu --timeout 120 --timeout-method thread -k "attention or fused_blocks or attn or keep_mask" > gpurun_out/r4_attn_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r4_attn_tests.log; [ $rc -eq 0 ] || exit $rc
: > gpurun_out/r4_attn_one.log
timeout -k 10 120 python tools/attn_one.py 0.1 20 2>&1 | grep -v amdgpu >> gpurun_out/r4_attn_one.log || exit 1
for km in 1 0 1 0; do for shp in 64,512,16 8,512,16; do echo "S=512 shape $shp" >> gpurun_out/r4_attn_one.log; ATTN_SHAPE=$shp ATTN_KMASK=$km timeout -k 10 120 python tools/attn_one.py 0.1 20 2>&1 | grep -v amdgpu >> gpurun_out/r4_attn_one.log || exit 1; done; done
cat gpurun_out/r4_attn_one.log
timeout -k 10 120 python tools/attn_phase_probe.py 0.1 > gpurun_out/attn_phase.jsonl 2>&1; rc=$?; grep -v amdgpu gpurun_out/attn_phase.jsonl; exit $rc
