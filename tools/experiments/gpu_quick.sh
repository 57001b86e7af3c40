# GEMM tests + seam probe + headline bench (one call)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_gemm.py > gpurun_out/gemm_tests.log 2>&1 || { tail -30 gpurun_out/gemm_tests.log; exit 1; }
tail -1 gpurun_out/gemm_tests.log
timeout -k 10 300 python tools/seam_probe.py > gpurun_out/seam_probe.log 2>&1 || { tail -20 gpurun_out/seam_probe.log; exit 1; }
cat gpurun_out/seam_probe.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench.log 2>&1 || { tail -20 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log | cut -c1-200
