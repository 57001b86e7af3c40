#!/bin/bash
# min-grid weight-gradient default: GEMM / e2e tests, bert-large S=512 B=8 and the headline
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_gemm.py tests/test_gpu_e2e.py > gpurun_out/mingrid_tests.log 2>&1 || { tail -30 gpurun_out/mingrid_tests.log; exit 1; }
tail -1 gpurun_out/mingrid_tests.log
timeout -k 10 300 python bench.py --model bert-large-uncased --seq_len 512 --batch_size 8 --steps 30 --warmup 5 2>/dev/null | tail -1 | cut -c1-100
timeout -k 10 300 python bench.py 2>/dev/null | tail -1 | cut -c1-100
