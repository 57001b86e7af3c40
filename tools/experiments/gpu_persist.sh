#!/bin/bash
# Persistent NT GEMM: bit-identity tests, per-GEMM A/B, headline bench A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_gemm.py -k "persistent" > gpurun_out/persist_test.log 2>&1 || { tail -30 gpurun_out/persist_test.log; exit 1; }
tail -2 gpurun_out/persist_test.log
timeout -k 10 300 python tools/env_ab_gemm.py HSD_G2_PERSIST 0,1 > gpurun_out/persist_ab.log 2>&1 || { tail -20 gpurun_out/persist_ab.log; exit 1; }
cat gpurun_out/persist_ab.log
CONFIGS="--batch_size 1024" bash tools/ab_env_bench.sh "HSD_G2_PERSIST=0" "HSD_G2_PERSIST=1" "HSD_G2_PERSIST=0" "HSD_G2_PERSIST=1"
