# fp8 weights re-quantised per optimizer slice under the backward (FusedAdam.per_slice_fp8) vs one pass at the end of
# the step: fp8 GPU tests + same-box MLM fp8 A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_fp8.py tests/test_gpu_e2e.py > gpurun_out/tests_f8slice.log 2>&1 || { tail -30 gpurun_out/tests_f8slice.log; exit 1; }
tail -2 gpurun_out/tests_f8slice.log
: > gpurun_out/f8slice_ab.log
for r in 1 2 3; do
  for v in True False; do
    timeout -k 10 300 python tools/bench_with.py optim.adam.FusedAdam.per_slice_fp8=$v -- --steps 8 --warmup 3 --model roberta-large --task masked-lm --seq_len 512 --batch_size 64 --dtype fp8 > gpurun_out/f8.json 2>gpurun_out/f8.err || { tail -20 gpurun_out/f8.err; exit 1; }
    tail -1 gpurun_out/f8.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('per_slice_fp8=$v roberta-large MLM B=64 fp8', d['value'], d['ms_per_step'])" | tee -a gpurun_out/f8slice_ab.log || exit 1
  done
done
