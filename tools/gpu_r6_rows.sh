# word-embedding Adam in two passes (untouched rows under the backward, the batch's rows after the embedding backward:
# LocalOverlap.two_pass_rows): GPU tests + same-box A/B at bert-large B=8 and the headline
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_e2e.py tests/test_gpu_graph.py tests/test_gpu_comm.py tests/test_gpu_ops.py -k "adam or optimizer or graph or comm or e2e" > gpurun_out/tests_rows.log 2>&1 || { tail -30 gpurun_out/tests_rows.log; exit 1; }
tail -2 gpurun_out/tests_rows.log
: > gpurun_out/rows_ab.log
for r in 1 2; do
  for v in True False; do
    for cfg in "--model bert-large-uncased --seq_len 512 --batch_size 8 --steps 30 --warmup 5" "--steps 10 --warmup 3"; do
      timeout -k 10 300 python tools/bench_with.py optim.adam.LocalOverlap.two_pass_rows=$v -- $cfg > gpurun_out/rw.json 2>gpurun_out/rw.err || { tail -20 gpurun_out/rw.err; exit 1; }
      tail -1 gpurun_out/rw.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('two_pass_rows=$v $cfg', d['value'], d['ms_per_step'])" | tee -a gpurun_out/rows_ab.log || exit 1
    done
  done
done
# weight-gradient grid at the headline (side stream): the cost model (0) vs min-grid plans of the 128 x 128 kernel
: > gpurun_out/wgrad_grid_ab.log
for r in 1 2; do
  for g in 0 192 256; do
    HSD_WGRAD_MIN_GRID=$g timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/wg.json 2>gpurun_out/wg.err || { tail -20 gpurun_out/wg.err; exit 1; }
    tail -1 gpurun_out/wg.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('HSD_WGRAD_MIN_GRID=$g headline', d['value'], d['ms_per_step'])" | tee -a gpurun_out/wgrad_grid_ab.log || exit 1
  done
done
