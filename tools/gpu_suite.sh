#!/bin/bash
# Full GPU tier (+ the 2-rank DP test rehearsed on one GPU over gloo) and the headline bench. Stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ${PYTEST_ARGS} > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -15 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
HSD_MULTIGPU_REHEARSE=1 timeout -k 10 300 python -u -m pytest tests/test_multigpu.py -x -q --timeout 280 --timeout-method thread > gpurun_out/multigpu_rehearse.log 2>&1
rc=$?; tail -3 gpurun_out/multigpu_rehearse.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench.log 2>&1 || { tail -20 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log
