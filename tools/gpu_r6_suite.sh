#!/bin/bash
# Round-6 GPU check: smoke, the whole GPU test tier, the headline bench; optional EXTRA command after them.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r6}
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_${TAG}.log 2>&1 || { tail -20 gpurun_out/smoke_${TAG}.log; exit 1; }
tail -1 gpurun_out/smoke_${TAG}.log
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 1500 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread ${PYTEST_ARGS} > gpurun_out/gpu_tests_${TAG}.log 2>&1
  rc=$?; tail -15 gpurun_out/gpu_tests_${TAG}.log
  [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_${TAG}.log 2>&1 || { tail -20 gpurun_out/bench_${TAG}.log; exit 1; }
tail -1 gpurun_out/bench_${TAG}.log | cut -c1-200
if [ -n "$EXTRA" ]; then bash -c "$EXTRA" || exit 1; fi
