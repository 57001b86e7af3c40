set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_gemm.py -x -q -k "schedules" --timeout 120 --timeout-method thread > gpurun_out/sched_tests.log 2>&1 || { tail -30 gpurun_out/sched_tests.log; exit 1; }
tail -3 gpurun_out/sched_tests.log
PROBE_SYNC=${PROBE_SYNC:-0,4,6,7} timeout -k 10 500 python -u tools/gemm_probe.py > gpurun_out/probe.log 2>&1 || { tail -30 gpurun_out/probe.log; exit 1; }
cat gpurun_out/probe.log
