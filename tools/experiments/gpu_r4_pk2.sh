#!/bin/bash
# gemm2pk2 (half-deferred epilogue persistent GEMM): bit-identity tests, per-GEMM A/B, bench A/B; attention tests and
# timing (bwd delta pre-pass reading dO from LDS).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_gemm.py -x -q --timeout 120 --timeout-method thread -k "half_deferred or gelu_derivative or persistent" > gpurun_out/r4_pk2_tests.log 2>&1
rc=$?; tail -5 gpurun_out/r4_pk2_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/env_ab_gemm.py HSD_G2_PK2 0,1 > gpurun_out/pk2_ab_r4.jsonl 2>&1 || { tail -20 gpurun_out/pk2_ab_r4.jsonl; exit 1; }
cat gpurun_out/pk2_ab_r4.jsonl
HSD_G2_PK2=1 timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r4_pk2_bench.log 2>&1 || { tail -20 gpurun_out/r4_pk2_bench.log; exit 1; }
tail -1 gpurun_out/r4_pk2_bench.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r4_pk_bench.log 2>&1 || { tail -20 gpurun_out/r4_pk_bench.log; exit 1; }
tail -1 gpurun_out/r4_pk_bench.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py -x -q -m gpu --timeout 120 --timeout-method thread -k "attention or fused_blocks" > gpurun_out/r4_attn_tests.log 2>&1
rc=$?; tail -5 gpurun_out/r4_attn_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python tools/attn_one.py 0.1 20 > gpurun_out/r4_attn_one.log 2>&1 && ATTN_SHAPE=64,512,16 timeout -k 10 120 python tools/attn_one.py 0.1 20 >> gpurun_out/r4_attn_one.log 2>&1
rc=$?; cat gpurun_out/r4_attn_one.log; exit $rc
