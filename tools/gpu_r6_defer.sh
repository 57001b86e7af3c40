# Adam slices ordered behind the next weight-gradient fork instead of their own compute-stream event
# (LocalOverlap.defer_to_fork): optimizer / e2e GPU tests + same-box A/B at bert-large B=8 and the headline
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_e2e.py tests/test_gpu_graph.py tests/test_gpu_comm.py > gpurun_out/tests_defer.log 2>&1 || { tail -30 gpurun_out/tests_defer.log; exit 1; }
tail -2 gpurun_out/tests_defer.log
: > gpurun_out/defer_ab.log
for v in True False True False; do
  for cfg in "--model bert-large-uncased --seq_len 512 --batch_size 8 --steps 30 --warmup 5" "--steps 10 --warmup 3"; do
    timeout -k 10 300 python tools/bench_with.py optim.adam.LocalOverlap.defer_to_fork=$v -- $cfg > gpurun_out/df.json 2>gpurun_out/df.err || { tail -20 gpurun_out/df.err; exit 1; }
    tail -1 gpurun_out/df.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('defer_to_fork=$v $cfg', d['value'], d['ms_per_step'])" | tee -a gpurun_out/defer_ab.log || exit 1
  done
done
