#!/bin/bash
# Round 5 pass T: LayerNorm fused into the persistent dropout + residual GEMM (gemm2_ln); tests + headline A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_gemm.py tests/test_gpu_ops.py tests/test_gpu_e2e.py -k "layernorm_tail or fused_blocks or persistent or hip_vs_reference" -x -q --timeout 300 --timeout-method thread > gpurun_out/ln_tail_tests.log 2>&1
rc=$?; tail -3 gpurun_out/ln_tail_tests.log; [ $rc -eq 0 ] || exit $rc
: > gpurun_out/ln_tail_ab.log
for r in 1 2 3; do
  for v in 0 1; do
    HSD_G2_LN=$v timeout -k 10 300 python bench.py --steps 20 --warmup 5 2>/dev/null | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('headline HSD_G2_LN=$v', d['value'], d['ms_per_step'])" | tee -a gpurun_out/ln_tail_ab.log || exit 1
  done
done
