#!/bin/bash
# One GPU round: build, GPU tests, bench, rocprofv3 kernel stats. Stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 900 python -m pytest tests -x -q -m gpu ${PYTEST_ARGS} > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -25 gpurun_out/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps ${STEPS:-20} --warmup 5 --batch_size ${BATCH:-1024} > gpurun_out/bench.log 2>&1 || { tail -20 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log
if [ -n "$PROFILE" ]; then
  rm -rf gpurun_out/prof
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python bench.py --steps 5 --warmup 3 --batch_size ${BATCH:-1024} > gpurun_out/prof.log 2>&1 || { tail -20 gpurun_out/prof.log; exit 1; }
  find gpurun_out/prof -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} gpurun_out/kernel_stats.csv
  head -40 gpurun_out/kernel_stats.csv | cut -c1-200
fi
