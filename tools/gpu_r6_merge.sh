# compute-stream events off the backward's critical path: Adam slices ordered behind the next weight-gradient fork
# (LocalOverlap.defer_to_fork) and one fork per block half for the weight gradients (hip._MERGE_FORKS): e2e / graph /
# comm / fp8 GPU tests + same-box A/B at bert-large B=8 and the headline
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_e2e.py tests/test_gpu_graph.py tests/test_gpu_comm.py tests/test_gpu_fp8.py > gpurun_out/tests_merge.log 2>&1 || { tail -30 gpurun_out/tests_merge.log; exit 1; }
tail -2 gpurun_out/tests_merge.log
: > gpurun_out/merge_ab.log
for r in 1 2; do
  for v in "True True" "False True" "False False"; do
    set -- $v
    for cfg in "--model bert-large-uncased --seq_len 512 --batch_size 8 --steps 30 --warmup 5" "--steps 10 --warmup 3"; do
      timeout -k 10 300 python tools/bench_with.py ops.hip._MERGE_FORKS=$1 optim.adam.LocalOverlap.defer_to_fork=$2 -- $cfg > gpurun_out/mf.json 2>gpurun_out/mf.err || { tail -20 gpurun_out/mf.err; exit 1; }
      tail -1 gpurun_out/mf.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('merge_forks=$1 defer_adam=$2 $cfg', d['value'], d['ms_per_step'])" | tee -a gpurun_out/merge_ab.log || exit 1
    done
  done
done
