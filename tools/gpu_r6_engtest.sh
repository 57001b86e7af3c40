# engine-path gradient zeroing test + the comm / e2e GPU tests
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_comm.py tests/test_gpu_e2e.py > gpurun_out/tests_eng.log 2>&1 || { tail -30 gpurun_out/tests_eng.log; exit 1; }
tail -2 gpurun_out/tests_eng.log
