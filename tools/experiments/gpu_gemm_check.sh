#!/bin/bash
# GEMM round: GEMM GPU tests, library comparison on the headline shapes, the headline bench. Stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_gemm.py -x -q --timeout 120 --timeout-method thread ${PYTEST_ARGS} > gpurun_out/gemm_tests.log 2>&1
rc=$?; tail -5 gpurun_out/gemm_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/vs_hipblaslt.py > gpurun_out/vs_hipblaslt.log 2>&1 || { tail -20 gpurun_out/vs_hipblaslt.log; exit 1; }
tail -1 gpurun_out/vs_hipblaslt.log | cut -c1-400
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench.log 2>&1 || { tail -20 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log
