#!/bin/bash
# gemm2pd (deferred-epilogue persistent GEMM): bit-identity tests, per-GEMM A/B, bench A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_gemm.py -x -q --timeout 120 --timeout-method thread -k "deferred or gelu_derivative" > gpurun_out/r4_pd_tests.log 2>&1
rc=$?; tail -5 gpurun_out/r4_pd_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/env_ab_gemm.py HSD_G2_PD 0,1 > gpurun_out/pd_ab_r4.jsonl 2>&1 && HSD_G2_PD=1 timeout -k 10 300 python -u tools/env_ab_gemm.py HSD_G2_GROUP 0,4,8,16 >> gpurun_out/pd_ab_r4.jsonl 2>&1 || { tail -20 gpurun_out/pd_ab_r4.jsonl; exit 1; }
cat gpurun_out/pd_ab_r4.jsonl
HSD_G2_PD=1 timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r4_pd_bench.log 2>&1 || { tail -20 gpurun_out/r4_pd_bench.log; exit 1; }
tail -1 gpurun_out/r4_pd_bench.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r4_pk_bench.log 2>&1 || { tail -20 gpurun_out/r4_pk_bench.log; exit 1; }
tail -1 gpurun_out/r4_pk_bench.log
