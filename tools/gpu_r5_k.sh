#!/bin/bash
# Round 5 pass K: attn128 backward at three workgroups per CU (V3) -- tests, kernel A/B, headline A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -k "attention" -x -q --timeout 120 --timeout-method thread > gpurun_out/attn_v3_tests.log 2>&1
rc=$?; tail -3 gpurun_out/attn_v3_tests.log; [ $rc -eq 0 ] || exit $rc
: > gpurun_out/attn_v3_ab.log
for v in 0 1 0 1; do
  HSD_A128_BWD_V3=$v timeout -k 10 120 python tools/attn_one.py 0.1 20 2>&1 | grep -v amdgpu.ids | sed "s/^/V3=$v /" | tee -a gpurun_out/attn_v3_ab.log || exit 1
done
for v in 0 1 0 1; do
  HSD_A128_BWD_V3=$v timeout -k 10 300 python bench.py --steps 20 --warmup 5 2>/dev/null | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('headline V3=$v', d['value'], d['ms_per_step'])" | tee -a gpurun_out/attn_v3_ab.log || exit 1
done
