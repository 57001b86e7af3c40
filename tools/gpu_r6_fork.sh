# stream-fork cost on the producer stream (tools/fork_cost.py)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 120 python tools/fork_cost.py 400 3 > gpurun_out/fork_cost.log 2>&1 || { tail -20 gpurun_out/fork_cost.log; exit 1; }
cat gpurun_out/fork_cost.log
timeout -k 10 120 python tools/fork_cost.py 400 20 >> gpurun_out/fork_cost.log 2>&1 || { tail -20 gpurun_out/fork_cost.log; exit 1; }
tail -6 gpurun_out/fork_cost.log
