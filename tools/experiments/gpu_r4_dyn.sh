#!/bin/bash
# Round-4 check of the dynamic tile queue: store-rate probe, GEMM tests, contention A/B, no-contention A/B, bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
hipcc --offload-arch=gfx950 -O3 -o /tmp/store_probe tools/store_probe.cpp || exit 1
timeout -k 10 120 /tmp/store_probe > gpurun_out/store_probe_r4.jsonl 2>&1 || { cat gpurun_out/store_probe_r4.jsonl; exit 1; }
cat gpurun_out/store_probe_r4.jsonl
timeout -k 10 600 python -u -m pytest tests/test_gpu_gemm.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r4_gemm_tests.log 2>&1
rc=$?; tail -5 gpurun_out/r4_gemm_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_gpu_fp32.py -x -q --timeout 180 --timeout-method thread > gpurun_out/r4_fp32_tests.log 2>&1
rc=$?; tail -15 gpurun_out/r4_fp32_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/contention_ab.py > gpurun_out/contention_ab_r4.jsonl 2>&1 || { tail -20 gpurun_out/contention_ab_r4.jsonl; exit 1; }
cat gpurun_out/contention_ab_r4.jsonl
timeout -k 10 300 python -u tools/env_ab_gemm.py HSD_G2_DYN 0,1 > gpurun_out/dyn_ab_r4.jsonl 2>&1 || { tail -20 gpurun_out/dyn_ab_r4.jsonl; exit 1; }
cat gpurun_out/dyn_ab_r4.jsonl
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r4_dyn_bench.log 2>&1 || { tail -20 gpurun_out/r4_dyn_bench.log; exit 1; }
tail -1 gpurun_out/r4_dyn_bench.log
HSD_G2_DYN=0 timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r4_static_bench.log 2>&1 || { tail -20 gpurun_out/r4_static_bench.log; exit 1; }
tail -1 gpurun_out/r4_static_bench.log
